// rvz_resnet.hip — the whole policy/value ResNet forward of the reference (network.py:30-117) in
// ONE gfx950 kernel per leaf batch, fp32 end to end on the f32-input MFMA (v_mfma_f32_32x32x2_f32,
// exact f32 FMA chains; the reference's precision).
//
// Why: with MIOpen, every conv layer is a separate launch plus a zero-fill of its output and a
// bias/skip/ReLU pass, and every activation makes an HBM round trip. Here a workgroup keeps its
// boards' activations in LDS for the whole network: HBM traffic is the leaf planes in and the
// logits/value out; weights stream from L2 (shared by every workgroup).
//
// Layout (one workgroup = 4 waves = NBOARD boards; F filters; 8x8 boards):
//   LDS act[2][NBOARD][64 pixels][F + 4 floats]   (ping-pong h / y; no halo: taps that leave the
//   board are masked to 0). A pixel row is F + 4 floats, so consecutive pixels start 4 banks apart.
//   conv layer = GEMM  M = NBOARD*64 pixels, N = F, K = 9 taps x F channels, on
//   v_mfma_f32_32x32x2_f32: A lane l = (pixel l&31 of a 32-pixel M-tile, k-slot l>>5), B lane l =
//   (k-slot l>>5, channel l&31 of the N-tile); k-slot h of step s is input channel h*(F/2)+s, so
//   one ds_read_b128 (A) / global_load_dwordx4 (B) feeds 4 steps. Every 16-lane group of a
//   ds_read_b128 then reads 16 distinct consecutive pixels: bank-conflict free (a 16x16x4 layout
//   mixed k-slots inside a group: 61% of its LDS cycles were conflicts, rocprof SQ_LDS_BANK_CONFLICT).
//   Wave w: N-tile, 2 M-tiles -> 2 accumulators of 16 floats.
// Packed parameter buffer (fp32, BN folded by rvz.LeafEvaluator; offsets in rvz_resnet_layout):
//   stem_w[F][27] (k = tap*3 + ch), stem_b[F], res_w[2NB][9][F(n)][F(k)], res_b[2NB][F],
//   pol_w[2][F], pol_b[2], pfc_w[65][128] (in = c*64 + px), pfc_b[65], val_w[F], val_b[1],
//   vfc1_w[256][64], vfc1_b[256], vfc2_w[256], vfc2_b[1].
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/rvz.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

struct Layout {
    int64_t stem_w, stem_b, res_w, res_b, pol_w, pol_b, pfc_w, pfc_b, val_w, val_b, vfc1_w,
        vfc1_b, vfc2_w, vfc2_b, total;
};

__host__ __device__ inline Layout make_layout(int F, int NB) {
    Layout L;
    int64_t o = 0;
    L.stem_w = o; o += (int64_t)F * 27;
    L.stem_b = o; o += F;
    o = (o + 3) & ~int64_t(3);
    L.res_w = o; o += (int64_t)2 * NB * 9 * F * F;
    L.res_b = o; o += (int64_t)2 * NB * F;
    L.pol_w = o; o += 2 * F;
    L.pol_b = o; o += 2;
    L.pfc_w = o; o += 65 * 128;
    L.pfc_b = o; o += 65;
    L.val_w = o; o += F;
    L.val_b = o; o += 1;
    L.vfc1_w = o; o += 256 * 64;
    L.vfc1_b = o; o += 256;
    L.vfc2_w = o; o += 256;
    L.vfc2_b = o; o += 1;
    L.total = o;
    return L;
}

template <int F, int NBOARD>
struct Cfg {
    static constexpr int CS = F + 4;                 // padded channel stride (bank spread)
    static constexpr int BOARD = 64 * CS;            // floats per board per buffer
    static constexpr int ACT = NBOARD * BOARD;       // floats per buffer
    static constexpr int XIN = NBOARD * 100 * 4;     // stem input, 3 planes padded to 4 (halo)
    static constexpr int HP = NBOARD * 128;          // policy conv output (NCHW flatten)
    static constexpr int HV = NBOARD * 64;           // value conv output
    static constexpr int H1 = NBOARD * 256;          // value fc1 output
    static constexpr int SMEM = 2 * ACT + XIN + HP + HV + H1;
    static constexpr int MTILES = 2 * NBOARD;        // 32-pixel M-tiles (4 board rows each)
    static constexpr int NTILES = F / 32;            // 32-channel N-tiles
    static_assert(MTILES * NTILES == 8, "8 tiles = 4 waves x 2 accumulators");
    static_assert(SMEM * 4 <= 160 * 1024, "fits the 160 KiB LDS of a CU");
};

typedef float f32x16 __attribute__((ext_vector_type(16)));

// One 3x3 conv layer: out = relu(conv(in) + bias (+ res)), all in LDS.
template <int F, int NBOARD, bool RES>
__device__ __forceinline__ void conv_layer(const float* __restrict__ in, float* __restrict__ out,
                                           const float* __restrict__ w,   // [9][F][F]
                                           const float* __restrict__ bias, int wave, int lane) {
    using C = Cfg<F, NBOARD>;
    constexpr int KH = F / 2;                     // steps per tap (2 k-slots)
    // wave -> (N-tile, first M-tile): F=64: 2 N-tiles x 4 M-tiles; F=128: 4 N-tiles x 2 M-tiles
    const int nt = F == 64 ? (wave & 1) : wave;
    const int mt0 = F == 64 ? 2 * (wave >> 1) : 0;
    const int h = lane >> 5, m = lane & 31;
    f32x16 acc0 = {}, acc1 = {};
    // A: pixel (mt*32 + m) of the workgroup; B: channel nt*32 + m
    const int pix0 = mt0 * 32 + m, pix1 = pix0 + 32;
    const int r0 = (pix0 & 63) >> 3, c0 = pix0 & 7, r1 = (pix1 & 63) >> 3, c1 = pix1 & 7;
    const float* brow = w + (size_t)(nt * 32 + m) * F + h * KH;
    const int koff = h * KH;
    for (int t = 0; t < 9; ++t) {
        const int dr = t / 3 - 1, dc = t % 3 - 1;
        const bool v0 = (unsigned)(r0 + dr) < 8u && (unsigned)(c0 + dc) < 8u;
        const bool v1 = (unsigned)(r1 + dr) < 8u && (unsigned)(c1 + dc) < 8u;
        // out-of-board taps read their own pixel and are zeroed (no halo in LDS)
        const float* a0p = in + (size_t)(v0 ? pix0 + dr * 8 + dc : pix0) * C::CS + koff;
        const float* a1p = in + (size_t)(v1 ? pix1 + dr * 8 + dc : pix1) * C::CS + koff;
        const float* bp = brow + (size_t)t * F * F;
#pragma unroll 4
        for (int g = 0; g < KH; g += 4) {
            const f32x4 bv = *reinterpret_cast<const f32x4*>(bp + g);
            f32x4 a0 = *reinterpret_cast<const f32x4*>(a0p + g);
            f32x4 a1 = *reinterpret_cast<const f32x4*>(a1p + g);
            if (!v0) a0 = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
            if (!v1) a1 = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[s], bv[s], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[s], bv[s], acc1, 0, 0, 0);
            }
        }
    }
    // epilogue: D col = lane&31 (channel), row = (reg&3) + 8*(reg>>2) + 4*(lane>>5) (pixel)
    const int n = nt * 32 + m;
    const float bn = bias[n];
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
        const int row = (reg & 3) + 8 * (reg >> 2) + 4 * h;
        const int o0 = (mt0 * 32 + row) * C::CS + n, o1 = o0 + 32 * C::CS;
        float x0 = acc0[reg] + bn, x1 = acc1[reg] + bn;
        if (RES) { x0 += out[o0]; x1 += out[o1]; }   // skip input h, read then overwritten in place
        out[o0] = fmaxf(x0, 0.0f);
        out[o1] = fmaxf(x1, 0.0f);
    }
}

template <int F, int NBOARD>
__global__ __launch_bounds__(256, 2) void k_resnet_fwd(const float* __restrict__ x, int n_boards,
                                                       const float* __restrict__ prm, Layout L,
                                                       int n_blocks, float* __restrict__ logits,
                                                       float* __restrict__ value) {
    using C = Cfg<F, NBOARD>;
    __shared__ __attribute__((aligned(16))) float smem[C::SMEM];
    float* actA = smem;
    float* actB = smem + C::ACT;
    float* xin = smem + 2 * C::ACT;
    float* hp = xin + C::XIN;
    float* hv = hp + C::HP;
    float* h1 = hv + C::HV;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g0 = blockIdx.x * NBOARD;

    // zero the stem input (its halo stays 0; the interior is written below)
    for (int i = tid; i < NBOARD * 100 * 4; i += 256) xin[i] = 0.0f;
    __syncthreads();
    for (int i = tid; i < NBOARD * 192; i += 256) {       // x[g][ch][r][c] -> xin[b][pad px][ch]
        const int b = i / 192, rem = i % 192, ch = rem / 64, px = rem % 64;
        const int g = g0 + b;
        const float v = g < n_boards ? x[(size_t)g * 192 + rem] : 0.0f;
        xin[(b * 100 + (px / 8 + 1) * 10 + (px % 8) + 1) * 4 + ch] = v;
    }
    __syncthreads();

    // stem: conv 3 -> F (VALU; 0.4% of the FLOPs), bias, ReLU -> actA
    {
        const int n = tid % F;
        float wv[27];
#pragma unroll
        for (int k = 0; k < 27; ++k) wv[k] = prm[L.stem_w + n * 27 + k];
        const float bn = prm[L.stem_b + n];
        for (int pi = tid / F; pi < NBOARD * 64; pi += 256 / F) {
            const int b = pi / 64, px = pi % 64, r = px / 8, c = px % 8;
            float acc = 0.0f;
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                const float* src = xin + (b * 100 + (r + t / 3) * 10 + (c + t % 3)) * 4;
#pragma unroll
                for (int ch = 0; ch < 3; ++ch) acc = fmaf(src[ch], wv[t * 3 + ch], acc);
            }
            actA[(b * 64 + px) * C::CS + n] = fmaxf(acc + bn, 0.0f);
        }
    }
    __syncthreads();

    for (int blk = 0; blk < n_blocks; ++blk) {
        const int l1 = 2 * blk, l2 = 2 * blk + 1;
        conv_layer<F, NBOARD, false>(actA, actB, prm + L.res_w + (size_t)l1 * 9 * F * F,
                                     prm + L.res_b + (size_t)l1 * F, wave, lane);
        __syncthreads();
        conv_layer<F, NBOARD, true>(actB, actA, prm + L.res_w + (size_t)l2 * 9 * F * F,
                                    prm + L.res_b + (size_t)l2 * F, wave, lane);
        __syncthreads();
    }

    // heads (network.py:104-117): 1x1 convs (BN folded) + ReLU
    for (int o = tid; o < NBOARD * 192; o += 256) {
        const int b = o / 192, rem = o % 192;
        const int c2 = rem / 64, px = rem % 64;            // c2 0,1: policy planes; 2: value
        const float* a = actA + (b * 64 + px) * C::CS;
        const float* wr = c2 < 2 ? prm + L.pol_w + c2 * F : prm + L.val_w;
        float acc = 0.0f;
        for (int k = 0; k < F; ++k) acc = fmaf(a[k], wr[k], acc);
        if (c2 < 2) hp[b * 128 + c2 * 64 + px] = fmaxf(acc + prm[L.pol_b + c2], 0.0f);
        else hv[b * 64 + px] = fmaxf(acc + prm[L.val_b], 0.0f);
    }
    __syncthreads();
    // policy fc (128 -> 65) and value fc1 (64 -> 256, ReLU)
    for (int o = tid; o < NBOARD * (65 + 256); o += 256) {
        const int b = o / 321, rem = o % 321;
        const int g = g0 + b;
        if (rem < 65) {
            const float* wr = prm + L.pfc_w + rem * 128;
            float acc = prm[L.pfc_b + rem];
            for (int i = 0; i < 128; ++i) acc = fmaf(hp[b * 128 + i], wr[i], acc);
            if (g < n_boards) logits[(size_t)g * 65 + rem] = acc;
        } else {
            const int u = rem - 65;
            const float* wr = prm + L.vfc1_w + u * 64;
            float acc = prm[L.vfc1_b + u];
            for (int i = 0; i < 64; ++i) acc = fmaf(hv[b * 64 + i], wr[i], acc);
            h1[b * 256 + u] = fmaxf(acc, 0.0f);
        }
    }
    __syncthreads();
    // value fc2 (256 -> 1) + tanh: one wave per board
    for (int b = wave; b < NBOARD; b += 4) {
        float acc = 0.0f;
        for (int i = lane; i < 256; i += 64) acc = fmaf(h1[b * 256 + i], prm[L.vfc2_w + i], acc);
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
        const int g = g0 + b;
        if (lane == 0 && g < n_boards) value[g] = tanhf(acc + prm[L.vfc2_b]);
    }
}

}  // namespace

extern "C" {

int64_t rvz_resnet_params_size(int32_t filters, int32_t blocks) {
    if ((filters != 64 && filters != 128) || blocks < 0) return RVZ_EINVAL;
    return make_layout(filters, blocks).total;
}

int rvz_resnet_fwd_f32(const float* x, int32_t n, const float* params, int32_t filters,
                       int32_t blocks, float* logits, float* value, void* stream) {
    if (!x || !params || !logits || !value || n < 0 || blocks < 0) return RVZ_EINVAL;
    if (((uintptr_t)params & 15) != 0) return RVZ_EINVAL;
    if (n == 0) return RVZ_OK;
    const Layout L = make_layout(filters, blocks);
    hipStream_t s = (hipStream_t)stream;
    if (filters == 64) {
        dim3 grid((n + 1) / 2), block(256);
        hipLaunchKernelGGL((k_resnet_fwd<64, 2>), grid, block, 0, s, x, n, params, L, blocks,
                           logits, value);
    } else if (filters == 128) {
        dim3 grid(n), block(256);
        hipLaunchKernelGGL((k_resnet_fwd<128, 1>), grid, block, 0, s, x, n, params, L, blocks,
                           logits, value);
    } else {
        return RVZ_EINVAL;
    }
    return hipGetLastError() == hipSuccess ? RVZ_OK : RVZ_EHIP;
}

}  // extern "C"
