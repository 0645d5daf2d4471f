// montecarlopathtracer_amd/csrc/box_quant.hpp driver:
//   box_quant_probe root.f32 in.f32 n out.u32
// root.f32 = bmin[3] bmax[3]; writes the grid (lo[3] sc[3] as float bits), then
// per input value v and axis a = i % 3 the code rounded down and the code
// rounded up.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../montecarlopathtracer_amd/csrc/box_quant.hpp"

int main(int argc, char** argv) {
    if (argc < 5) return 2;
    float root[6];
    FILE* fp = std::fopen(argv[1], "rb");
    if (!fp || std::fread(root, 4, 6, fp) != 6) return 1;
    std::fclose(fp);
    const long n = std::atol(argv[3]);
    std::vector<float> x(n);
    fp = std::fopen(argv[2], "rb");
    if (!fp || std::fread(x.data(), 4, n, fp) != size_t(n)) return 1;
    std::fclose(fp);
    const mcpt::BoxGrid g = mcpt::box_grid(root, root + 3);
    std::vector<uint32_t> out(6 + 2 * n);
    std::memcpy(out.data(), g.lo, 12);
    std::memcpy(out.data() + 3, g.sc, 12);
    for (long i = 0; i < n; ++i) {
        out[6 + 2 * i] = mcpt::box_q_down(g, int(i % 3), x[i]);
        out[6 + 2 * i + 1] = mcpt::box_q_up(g, int(i % 3), x[i]);
    }
    fp = std::fopen(argv[4], "wb");
    if (!fp) return 1;
    std::fwrite(out.data(), 4, out.size(), fp);
    std::fclose(fp);
    std::printf("ok\n");
    return 0;
}
