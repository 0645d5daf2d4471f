// math_probe.hip -- test-only probe of the product's device math
// (montecarlopathtracer_amd/csrc/mcpt_device.hpp) for bitwise comparison with
// the CPU specification (oracle).  Built by tests/hip/build_probe.py.
#include <hip/hip_runtime.h>
#include "../../montecarlopathtracer_amd/csrc/mcpt_device.hpp"

using namespace mcpt::dev;

__global__ void probe(int op, int n, const float* a, const float* b, float* o0, float* o1, uint32_t* u) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float x = a[i], y = b[i];
    switch (op) {
        case 0: o0[i] = x / y; break;
        case 1: o0[i] = 1.0f / x; break;
        case 2: o0[i] = sqrt_rn(x); break;
        case 3: { float s, c; sincos_f(x, s, c); o0[i] = s; o1[i] = c; } break;
        case 4: o0[i] = pow_f(x, y); break;
        case 5: { double q = (double)x / (double)y; uint64_t bits = __builtin_bit_cast(uint64_t, q);
                  u[2 * i] = (uint32_t)bits; u[2 * i + 1] = (uint32_t)(bits >> 32); } break;
        case 6: { uint32_t sd = rng_init((uint32_t)i, __float_as_uint(x), __float_as_uint(y));
                  u[2 * i] = sd; o0[i] = rng_next(sd); u[2 * i + 1] = sd; } break;
        case 7: { V3 n = v3(x, y, 0.3f); normalize_cu(n); o0[i] = n.x; o1[i] = n.y; } break;
        case 8: { float t = (x - y) * (1.0f / (y - 0.5f)); o0[i] = t; } break;
        case 9: o0[i] = sqrtf(x); break;
        case 10: o0[i] = __builtin_sqrtf(x); break;
        case 11: o0[i] = pow5_f(x); break;
        case 12: o0[i] = (float)((double)x * (1.0 / (double)y)); break;
        case 13: { const double d = (double)y, r0 = __builtin_amdgcn_rcp(d);
                   double e = __builtin_fma(-d, r0, 1.0); const double r1 = __builtin_fma(r0, e, r0);
                   e = __builtin_fma(-d, r1, 1.0); const double r2 = __builtin_fma(r1, e, r1);
                   o0[i] = (float)((double)x * ((__builtin_isfinite(r0) && r0 != 0.0) ? r2 : r0)); } break;
        default: break;
    }
}

extern "C" int math_probe(int op, int n, const float* a, const float* b, float* o0, float* o1, uint32_t* u) {
    float *da, *db, *d0, *d1; uint32_t* du;
    size_t fb = sizeof(float) * (size_t)n;
    if (hipMalloc(&da, fb) || hipMalloc(&db, fb) || hipMalloc(&d0, fb) || hipMalloc(&d1, fb) ||
        hipMalloc(&du, 2 * sizeof(uint32_t) * (size_t)n)) return -1;
    hipMemcpy(da, a, fb, hipMemcpyHostToDevice);
    hipMemcpy(db, b, fb, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3((n + 255) / 256), dim3(256), 0, 0, op, n, da, db, d0, d1, du);
    hipError_t e = hipDeviceSynchronize();
    hipMemcpy(o0, d0, fb, hipMemcpyDeviceToHost);
    hipMemcpy(o1, d1, fb, hipMemcpyDeviceToHost);
    hipMemcpy(u, du, 2 * sizeof(uint32_t) * (size_t)n, hipMemcpyDeviceToHost);
    hipFree(da); hipFree(db); hipFree(d0); hipFree(d1); hipFree(du);
    return e == hipSuccess ? 0 : -2;
}
