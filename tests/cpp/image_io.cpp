// include/mcpt_image_io.hpp driver: image_io in.f32 W H out.u8 out.png out.pfm
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "mcpt_image_io.hpp"

int main(int argc, char** argv) {
    if (argc < 7) return 2;
    const int W = std::atoi(argv[2]), H = std::atoi(argv[3]);
    std::vector<float> rgb(size_t(W) * H * 3);
    FILE* fp = std::fopen(argv[1], "rb");
    if (!fp || std::fread(rgb.data(), sizeof(float), rgb.size(), fp) != rgb.size()) return 1;
    std::fclose(fp);
    const std::vector<uint8_t> e = mcpt::image::encode_8bit_cv(rgb.data(), W, H);
    fp = std::fopen(argv[4], "wb");
    if (!fp) return 1;
    std::fwrite(e.data(), 1, e.size(), fp);
    std::fclose(fp);
    if (!mcpt::image::write_png(argv[5], rgb.data(), W, H)) return 1;
    if (!mcpt::image::write_pfm(argv[6], rgb.data(), W, H)) return 1;
    std::printf("ok\n");
    return 0;
}
