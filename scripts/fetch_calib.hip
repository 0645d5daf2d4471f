// fetch_calib.hip -- calibration of the L2 fabric-read counters on gfx950
// for the access patterns of the wavefront extend.
//
// Known byte counts, each kernel launched once per pass:
//   calib_stream          a 1 GiB buffer read once, 16 B per lane, coalesced
//                         (the guide's case: FETCH_SIZE reports half of it)
//   calib_gather<128, 0>  N 48-B records, each alone at the start of its own
//                         128-B line, each read once in a random order (3 x 16-B
//                         loads per lane): N distinct lines, 48 B of each
//   calib_gather<128, 40> the same with the record at byte 40 of its line (it
//                         straddles the line's two 64-B halves)
//   calib_gather<48, 0>   N packed 48-B records (the C4 pair-record layout)
//                         each read once in a random order
// plus the permutation's own 4-B-per-lane stream.  Run under rocprofv3 --pmc
// with FETCH_SIZE, or with TCC_EA0_RDREQ{,_32B,_64B,_128B}, or with
// TCC_EA0_RDREQ_DRAM{,_32B} TCC_BUBBLE (scripts/fetch_calib.sh), and compare
// each counter's bytes with the known ones (scripts/fetch_calib_report.py).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                        \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                               \
        }                                                                               \
    } while (0)

__global__ void __launch_bounds__(256) calib_stream(const uint4* __restrict__ src, size_t n16, uint32_t* out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256ull) {
        const uint4 v = src[i];
        acc ^= v.x + v.y + v.z + v.w;
    }
    out[blockIdx.x * 256u + threadIdx.x] = acc;
}

template <int STRIDE, int OFF>
__global__ void __launch_bounds__(256) calib_gather(const unsigned char* __restrict__ buf,
                                                    const uint32_t* __restrict__ perm, uint32_t n, uint32_t* out) {
    uint32_t acc = 0;
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
        const uint4* r = reinterpret_cast<const uint4*>(buf + (size_t)perm[i] * STRIDE + OFF);
        const uint4 a = r[0], b = r[1], c = r[2];
        acc ^= a.x + b.y + c.z + a.w + b.x + c.y;
    }
    out[blockIdx.x * 256u + threadIdx.x] = acc;
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)std::atoi(argv[1]) : (1u << 20);   // records per gather
    const size_t stream_bytes = size_t(1) << 30;
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int grid = cus * 8;
    unsigned char *sbuf = nullptr, *gbuf = nullptr;
    uint32_t *perm = nullptr, *out = nullptr;
    const size_t gbytes = size_t(n) * 128 + 256;
    CHECK(hipMalloc(&sbuf, stream_bytes));
    CHECK(hipMalloc(&gbuf, gbytes));
    CHECK(hipMalloc(&perm, size_t(n) * 4));
    CHECK(hipMalloc(&out, size_t(grid) * 256 * 4));
    CHECK(hipMemset(sbuf, 1, stream_bytes));
    CHECK(hipMemset(gbuf, 2, gbytes));
    std::vector<uint32_t> p(n);
    for (uint32_t i = 0; i < n; i++) p[i] = i;
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (uint32_t i = n - 1; i > 0; i--) {   // Fisher-Yates with a fixed xorshift stream
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        const uint32_t j = (uint32_t)(x % (i + 1));
        std::swap(p[i], p[j]);
    }
    CHECK(hipMemcpy(perm, p.data(), size_t(n) * 4, hipMemcpyHostToDevice));
    // evict the L2s / Infinity Cache between kernels: stream a 512 MiB scratch write
    unsigned char* flush = nullptr;
    CHECK(hipMalloc(&flush, size_t(512) << 20));
    auto evict = [&]() { CHECK(hipMemsetAsync(flush, 3, size_t(512) << 20, 0)); };
    evict();
    hipLaunchKernelGGL(calib_stream, dim3(grid), dim3(256), 0, 0, reinterpret_cast<const uint4*>(sbuf),
                       stream_bytes / 16, out);
    evict();
    hipLaunchKernelGGL((calib_gather<128, 0>), dim3(grid), dim3(256), 0, 0, gbuf, perm, n, out);
    evict();
    hipLaunchKernelGGL((calib_gather<128, 40>), dim3(grid), dim3(256), 0, 0, gbuf, perm, n, out);
    evict();
    hipLaunchKernelGGL((calib_gather<48, 0>), dim3(grid), dim3(256), 0, 0, gbuf, perm, n, out);
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    std::printf("{\"records\": %u, \"stream_bytes\": %zu, \"record_bytes\": 48, \"perm_bytes\": %zu, \"grid\": %d}\n",
                n, stream_bytes, size_t(n) * 4, grid);
    CHECK(hipFree(flush));
    CHECK(hipFree(sbuf));
    CHECK(hipFree(gbuf));
    CHECK(hipFree(perm));
    CHECK(hipFree(out));
    return 0;
}
