// QuinEngine viewer loop through include/mcpt_qe_viewer.hpp (GraphicsRTX::DoOnUpdate).
// usage: qe_viewer scene.obj W H frames screen.bin saved.png [tinyobj|cvmctracer]
// prints the frame seeds it drew, writes the final screen (float RGB) and the
// PNG the viewer saved every `frames` frames.
#include <cstdio>
#include <cstdlib>
#include <string>

#include "mcpt_qe_viewer.hpp"

int main(int argc, char** argv) {
    if (argc < 7) return 2;
    const uint32_t W = std::atoi(argv[2]), H = std::atoi(argv[3]);
    const int frames = std::atoi(argv[4]);
    const int32_t flavor = (argc > 7 && std::string(argv[7]) == "cvmctracer") ? MCPT_OBJ_CVMCTRACER : MCPT_OBJ_TINYOBJ;
    mcpt::qe::Viewer v;
    if (v.Initialize(argv[1], W, H, 0, flavor) != MCPT_OK) { std::printf("init failed: %s\n", mcpt_last_error()); return 1; }
    v.SetSaveEvery(frames, argv[6]);
    for (int f = 0; f < frames; ++f) {
        if (v.OnUpdate() != MCPT_OK) { std::printf("frame failed: %s\n", mcpt_last_error()); return 1; }
        std::printf("seed %u\n", v.LastSeed());
    }
    FILE* fp = std::fopen(argv[5], "wb");
    if (!fp) return 1;
    std::fwrite(v.Screen(), sizeof(float), size_t(W) * H * 3, fp);
    std::fclose(fp);
    v.Shutdown();
    std::printf("ok %u\n", v.Frames());
    return 0;
}
