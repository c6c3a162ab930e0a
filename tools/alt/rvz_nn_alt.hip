// rvz_nn_alt.hip (tools/alt/librvz_alt.so, the MIOpen evaluator's A/B path) — leaf-evaluator helpers for the policy/value ResNet.
//
// MIOpen's NHWC fp32 implicit-GEMM convolution runs at ~85% of the fp32 MFMA peak on the C2 shape,
// but PyTorch then spends three more full passes over every activation: the conv bias add, the
// ReLU and the residual add (network.py:23-28,97). This kernel does all three in one in-place
// pass over the conv output (BN is folded into the conv weights/bias by rvz.LeafEvaluator):
//     x = relu(x + bias[c] (+ residual))
// x / residual are NHWC (channels_last) tensors of n_pix pixels x C channels, C % 4 == 0.
#include <hip/hip_bf16.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rvz_alt.h"

namespace {

template <bool RES, bool RELU>
__global__ __launch_bounds__(256) void k_bias_act_f32(float4* __restrict__ x,
                                                      const float4* __restrict__ bias,
                                                      const float4* __restrict__ res,
                                                      int64_t n_vec, int c_vec) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_vec; i += stride) {
        float4 v = x[i];
        const float4 b = bias[i % c_vec];
        v.x += b.x; v.y += b.y; v.z += b.z; v.w += b.w;
        if (RES) {
            const float4 r = res[i];
            v.x += r.x; v.y += r.y; v.z += r.z; v.w += r.w;
        }
        if (RELU) {
            v.x = fmaxf(v.x, 0.0f); v.y = fmaxf(v.y, 0.0f);
            v.z = fmaxf(v.z, 0.0f); v.w = fmaxf(v.w, 0.0f);
        }
        x[i] = v;
    }
}

// bf16 activations, f32 bias: 8 elements (16 B) per thread; the sum is rounded to bf16 once.
template <bool RES, bool RELU>
__global__ __launch_bounds__(256) void k_bias_act_bf16(uint4* __restrict__ x,
                                                       const float* __restrict__ bias,
                                                       const uint4* __restrict__ res,
                                                       int64_t n_vec, int channels) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_vec; i += stride) {
        uint4 v = x[i];
        uint4 r = RES ? res[i] : make_uint4(0, 0, 0, 0);
        const int c0 = (int)((i * 8) % channels);
        uint32_t* vw = reinterpret_cast<uint32_t*>(&v);
        const uint32_t* rw = reinterpret_cast<const uint32_t*>(&r);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float lo = __uint_as_float(vw[k] << 16) + bias[c0 + 2 * k];
            float hi = __uint_as_float(vw[k] & 0xffff0000u) + bias[c0 + 2 * k + 1];
            if (RES) {
                lo += __uint_as_float(rw[k] << 16);
                hi += __uint_as_float(rw[k] & 0xffff0000u);
            }
            if (RELU) { lo = fmaxf(lo, 0.0f); hi = fmaxf(hi, 0.0f); }
            const __hip_bfloat16 blo = __float2bfloat16(lo), bhi = __float2bfloat16(hi);
            vw[k] = (uint32_t)(*reinterpret_cast<const uint16_t*>(&blo)) |
                    ((uint32_t)(*reinterpret_cast<const uint16_t*>(&bhi)) << 16);
        }
        x[i] = v;
    }
}

int grid_for(int64_t n_vec) {
    int64_t g = (n_vec + 255) / 256;
    return (int)(g < 2048 ? (g > 0 ? g : 1) : 2048);   // 256 CUs x 8: grid-stride the rest
}

}  // namespace

extern "C" {

int rvz_nn_bias_act_f32(float* x, const float* bias, const float* residual, int64_t n_pix,
                        int32_t channels, int32_t relu, void* stream) {
    if (!x || !bias || n_pix < 0 || channels <= 0 || channels % 4) return RVZ_EINVAL;
    if (((uintptr_t)x | (uintptr_t)bias | (uintptr_t)residual) & 15) return RVZ_EINVAL;
    const int64_t n_vec = n_pix * channels / 4;
    if (n_vec == 0) return RVZ_OK;
    const int cv = channels / 4;
    hipStream_t s = (hipStream_t)stream;
    float4* xv = reinterpret_cast<float4*>(x);
    const float4* bv = reinterpret_cast<const float4*>(bias);
    const float4* rv = reinterpret_cast<const float4*>(residual);
    dim3 grid(grid_for(n_vec)), block(256);
    if (residual && relu) hipLaunchKernelGGL((k_bias_act_f32<true, true>), grid, block, 0, s, xv, bv, rv, n_vec, cv);
    else if (residual) hipLaunchKernelGGL((k_bias_act_f32<true, false>), grid, block, 0, s, xv, bv, rv, n_vec, cv);
    else if (relu) hipLaunchKernelGGL((k_bias_act_f32<false, true>), grid, block, 0, s, xv, bv, rv, n_vec, cv);
    else hipLaunchKernelGGL((k_bias_act_f32<false, false>), grid, block, 0, s, xv, bv, rv, n_vec, cv);
    return hipGetLastError() == hipSuccess ? RVZ_OK : RVZ_EHIP;
}

int rvz_nn_bias_act_bf16(void* x, const float* bias, const void* residual, int64_t n_pix,
                         int32_t channels, int32_t relu, void* stream) {
    if (!x || !bias || n_pix < 0 || channels <= 0 || channels % 8) return RVZ_EINVAL;
    if (((uintptr_t)x | (uintptr_t)residual) & 15) return RVZ_EINVAL;
    const int64_t n_vec = n_pix * channels / 8;
    if (n_vec == 0) return RVZ_OK;
    hipStream_t s = (hipStream_t)stream;
    uint4* xv = reinterpret_cast<uint4*>(x);
    const uint4* rv = reinterpret_cast<const uint4*>(residual);
    dim3 grid(grid_for(n_vec)), block(256);
    if (residual && relu) hipLaunchKernelGGL((k_bias_act_bf16<true, true>), grid, block, 0, s, xv, bias, rv, n_vec, channels);
    else if (residual) hipLaunchKernelGGL((k_bias_act_bf16<true, false>), grid, block, 0, s, xv, bias, rv, n_vec, channels);
    else if (relu) hipLaunchKernelGGL((k_bias_act_bf16<false, true>), grid, block, 0, s, xv, bias, rv, n_vec, channels);
    else hipLaunchKernelGGL((k_bias_act_bf16<false, false>), grid, block, 0, s, xv, bias, rv, n_vec, channels);
    return hipGetLastError() == hipSuccess ? RVZ_OK : RVZ_EHIP;
}

}  // extern "C"
