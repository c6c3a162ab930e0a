// rvz_numerics_alt.hip (tools/alt/librvz_alt.so) — the engine's scalar numerics as standalone
// kernels, compiled with the product's flags, so tests/test_gpu_numerics.py can check them
// against NumPy element by element: sqrt_count (csrc/rvz_engine.hip) = np.float32(math.sqrt(n)).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rvz_alt.h"

namespace {
// the same expression as csrc/rvz_engine.hip sqrt_count
__device__ __forceinline__ float sqrt_count(int n) { return __builtin_sqrtf((float)n); }

__global__ void k_sqrt_count(int n, float* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = sqrt_count(i);
}
}  // namespace

extern "C" int rvz_alt_sqrt_count(int32_t n, float* out, void* stream) {
    if (n < 0 || (n > 0 && !out)) return RVZ_EINVAL;
    if (n == 0) return RVZ_OK;
    hipLaunchKernelGGL(k_sqrt_count, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, n,
                       out);
    return hipGetLastError() == hipSuccess ? RVZ_OK : RVZ_EHIP;
}
