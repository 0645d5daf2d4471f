// montecarlopathtracer_amd/csrc/half_box.hpp driver: half_box_probe in.f32 n out.u16
// writes, per input, the fp16 rounded down then the fp16 rounded up.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../montecarlopathtracer_amd/csrc/half_box.hpp"

int main(int argc, char** argv) {
    if (argc < 4) return 2;
    const long n = std::atol(argv[2]);
    std::vector<float> x(n);
    FILE* fp = std::fopen(argv[1], "rb");
    if (!fp || std::fread(x.data(), 4, n, fp) != size_t(n)) return 1;
    std::fclose(fp);
    std::vector<uint16_t> out(2 * n);
    for (long i = 0; i < n; ++i) {
        out[2 * i] = mcpt::f32_to_f16_dir(x[i], -1);
        out[2 * i + 1] = mcpt::f32_to_f16_dir(x[i], +1);
    }
    fp = std::fopen(argv[3], "wb");
    if (!fp) return 1;
    std::fwrite(out.data(), 2, out.size(), fp);
    std::fclose(fp);
    std::printf("ok\n");
    return 0;
}
