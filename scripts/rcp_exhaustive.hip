// Exhaustive check (every binary32 bit pattern) of an FMA-corrected hardware
// reciprocal against IEEE 1.0f / b on this GPU:
//   y0 = v_rcp_f32(b); e = fma(-b, y0, 1); y1 = fma(e, y0, y0)
// with b = +-0 / +-inf / NaN passed through as v_rcp_f32's own result.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off scripts/rcp_exhaustive.hip -o /tmp/rcp_x
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>

__device__ __forceinline__ float rcp_nr(float b) {
    const float y0 = __builtin_amdgcn_rcpf(b);
    const float e = __builtin_fmaf(-b, y0, 1.0f);
    const float y1 = __builtin_fmaf(e, y0, y0);
    return (__builtin_isfinite(y0) && y0 != 0.0f) ? y1 : y0;
}

// mode 0: every pattern; 1: only 2^-126 <= |b| < 2^126 (normal b, normal 1/b)
__global__ void check(uint64_t base, unsigned long long* bad, uint32_t* first, int mode) {
    const uint64_t i = base + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t u = (uint32_t)i;
    const float b = __uint_as_float(u);
    const uint32_t ex = (u >> 23) & 0xFFu;
    if (mode == 1 && (ex < 1u || ex >= 253u)) return;
    const float ref = 1.0f / b;
    const float got = rcp_nr(b);
    const bool same = (__float_as_uint(ref) == __float_as_uint(got)) || (ref != ref && got != got);
    if (!same) {
        const unsigned long long k = atomicAdd(bad, 1ull);
        if (k < 16) first[k] = u;
    }
}

int main() {
    unsigned long long* bad;
    uint32_t* first;
    hipMalloc(&bad, 8);
    hipMalloc(&first, 64);
    for (int mode = 1; mode >= 0; mode--) {
    hipMemset(bad, 0, 8);
    hipMemset(first, 0, 64);
    const uint64_t chunk = 1ull << 28;
    for (uint64_t base = 0; base < (1ull << 32); base += chunk) {
        hipLaunchKernelGGL(check, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, base, bad, first, mode);
    }
    unsigned long long nb = 0;
    uint32_t f[16];
    hipMemcpy(&nb, bad, 8, hipMemcpyDeviceToHost);
    hipMemcpy(f, first, 64, hipMemcpyDeviceToHost);
    printf("mode %d: mismatches %llu\n", mode, nb);
    for (int k = 0; k < 16 && k < (int)nb; k++) {
        float x;
        memcpy(&x, &f[k], 4);
        printf("  0x%08x  %.9g\n", f[k], x);
    }
    }
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
