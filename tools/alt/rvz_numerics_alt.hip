// rvz_numerics_alt.hip (tools/alt/librvz_alt.so) — the engine's scalar numerics as standalone
// kernels, compiled with the product's flags, so tests/test_gpu_numerics.py can check them
// against NumPy element by element: sqrt_count (csrc/rvz_engine.hip) = np.float32(math.sqrt(n)),
// and k_act's power (csrc/rvz_pow.hip.h pow_cr, on the device and on the host; mode 0 = the device
// library's pow, for comparison).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../alphazero-reversi_amd/csrc/rvz_pow.hip.h"
#include "rvz_alt.h"

namespace {
// the same expression as csrc/rvz_engine.hip sqrt_count
__device__ __forceinline__ float sqrt_count(int n) { return __builtin_sqrtf((float)n); }

__global__ void k_sqrt_count(int n, float* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = sqrt_count(i);
}

__global__ void k_pow(int n, const double* __restrict__ x, const double* __restrict__ e,
                      double* __restrict__ out, int mode) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = mode ? rvz_pow::pow_cr(x[i], e[i]) : pow(x[i], e[i]);
}
}  // namespace

extern "C" int rvz_alt_pow(int32_t n, const double* x, const double* e, double* out, int32_t mode,
                           void* stream) {
    if (n < 0 || (n > 0 && (!x || !e || !out))) return RVZ_EINVAL;
    if (n == 0) return RVZ_OK;
    hipLaunchKernelGGL(k_pow, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, n, x, e,
                       out, mode);
    return hipGetLastError() == hipSuccess ? RVZ_OK : RVZ_EHIP;
}

extern "C" int rvz_alt_pow_host(int32_t n, const double* x, const double* e, double* out) {
    if (n < 0 || (n > 0 && (!x || !e || !out))) return RVZ_EINVAL;
    for (int32_t i = 0; i < n; ++i) out[i] = rvz_pow::pow_cr(x[i], e[i]);
    return RVZ_OK;
}

extern "C" int rvz_alt_sqrt_count(int32_t n, float* out, void* stream) {
    if (n < 0 || (n > 0 && !out)) return RVZ_EINVAL;
    if (n == 0) return RVZ_OK;
    hipLaunchKernelGGL(k_sqrt_count, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, n,
                       out);
    return hipGetLastError() == hipSuccess ? RVZ_OK : RVZ_EHIP;
}
