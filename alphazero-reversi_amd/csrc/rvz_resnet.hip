// rvz_resnet.hip — the whole policy/value ResNet forward of the reference (network.py:30-117) in
// ONE gfx950 kernel per leaf batch, fp32 end to end on the f32-input MFMA (v_mfma_f32_16x16x4_f32,
// exact f32 FMA chains; the reference's precision).
//
// Why: with MIOpen, every conv layer is a separate launch plus a zero-fill of its output and a
// bias/skip/ReLU pass, and every activation makes an HBM round trip. Here a workgroup keeps its
// boards' activations in LDS for the whole network: HBM traffic is the leaf planes in and the
// logits/value out; weights stream from L2 (shared by every workgroup).
//
// Layout (one workgroup = 4 waves = NBOARD boards; F filters; 8x8 boards):
//   LDS act[2][NBOARD][10x10 padded pixels][F + 4 floats]   (ping-pong h / y, zero halo)
//   conv layer = GEMM  M = NBOARD*64 pixels, N = F, K = 9 taps x F channels.
//   MFMA 16x16x4: A lane l = (pixel l&15 of the M-tile, k-slot l>>4), B lane l = (k-slot l>>4,
//   channel l&15 of the N-tile). k-slot q of step s of tap t is input channel q*(F/4)+s, so one
//   ds_read_b128 (A) / global_load_dwordx4 (B) feeds 4 consecutive steps.
//   Wave w owns N-tiles {w, w+4, ..} and every M-tile: MT*NT = 8 accumulators of 4 floats.
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
    static constexpr int BOARD = 100 * CS;           // floats per board per buffer
    static constexpr int ACT = NBOARD * BOARD;       // floats per buffer
    static constexpr int XIN = NBOARD * 100 * 4;     // stem input, 3 planes padded to 4
    static constexpr int HP = NBOARD * 128;          // policy conv output (NCHW flatten)
    static constexpr int HV = NBOARD * 64;           // value conv output
    static constexpr int H1 = NBOARD * 256;          // value fc1 output
    static constexpr int SMEM = 2 * ACT + XIN + HP + HV + H1;
    static constexpr int MT = 4 * NBOARD;            // 16-pixel M-tiles (2 board rows each)
    static constexpr int NT = F / 64;                // N-tiles per wave
    static_assert(MT * NT == 8, "8 accumulators per wave");
    static_assert(SMEM * 4 <= 160 * 1024, "fits the 160 KiB LDS of a CU");
};

// padded pixel index of M-tile row p (0..15) of tile mt, shifted by tap t
__device__ __forceinline__ int tile_pix(int mt, int p, int t) {
    const int b = mt >> 2, tr = mt & 3;
    const int r = 2 * tr + (p >> 3), c = p & 7;
    const int dr = t / 3 - 1, dc = t % 3 - 1;
    return b * 100 + (r + 1 + dr) * 10 + (c + 1 + dc);
}

// One 3x3 conv layer: out = relu(conv(in) + bias (+ res)), all in LDS.
template <int F, int NBOARD, bool RES>
__device__ __forceinline__ void conv_layer(const float* __restrict__ in, float* __restrict__ out,
                                           const float* __restrict__ w,   // [9][F][F]
                                           const float* __restrict__ bias, int wave, int lane) {
    using C = Cfg<F, NBOARD>;
    constexpr int MT = C::MT, NT = C::NT, KQ = F / 4;   // steps per tap
    const int q = lane >> 4, p = lane & 15;
    f32x4 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    // per-lane base addresses: A at (pixel, channel q*KQ), B at (channel n, k q*KQ)
    int abase[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) abase[i] = tile_pix(i, p, 4) * C::CS + q * KQ;   // tap 4 = center
    const float* bbase[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) bbase[j] = w + (size_t)((wave + 4 * j) * 16 + p) * F + q * KQ;
    // K loop over 9 taps x KQ/4 groups of 4 steps, software-pipelined one group deep: the next
    // group's weight (global/L2) and activation (LDS) operands load under this group's MFMAs.
    constexpr int GPT = KQ / 4;          // groups per tap
    constexpr int NG = 9 * GPT;
    f32x4 a_cur[MT], b_cur[NT], a_nxt[MT], b_nxt[NT];
    auto load = [&](int it, f32x4* av, f32x4* bv) {
        const int t = it / GPT, g = (it % GPT) * 4;
        const int shift = ((t / 3 - 1) * 10 + (t % 3 - 1)) * C::CS;   // tap offset in LDS
#pragma unroll
        for (int j = 0; j < NT; ++j)
            bv[j] = *reinterpret_cast<const f32x4*>(bbase[j] + (size_t)t * F * F + g);
#pragma unroll
        for (int i = 0; i < MT; ++i)
            av[i] = *reinterpret_cast<const f32x4*>(in + abase[i] + shift + g);
    };
    load(0, a_cur, b_cur);
    for (int it = 0; it < NG; ++it) {
        if (it + 1 < NG) load(it + 1, a_nxt, b_nxt);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int j = 0; j < NT; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a_cur[i][s], b_cur[j][s],
                                                                    acc[i][j], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < MT; ++i) a_cur[i] = a_nxt[i];
#pragma unroll
        for (int j = 0; j < NT; ++j) b_cur[j] = b_nxt[j];
    }
    // epilogue: D row = (lane>>4)*4 + r (pixel in the tile), col = lane&15 (channel in the tile)
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int n = (wave + 4 * j) * 16 + p;
        const float bn = bias[n];
#pragma unroll
        for (int i = 0; i < MT; ++i) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int off = tile_pix(i, 4 * q + r, 4) * C::CS + n;
                float v = acc[i][j][r] + bn;
                if (RES) v += out[off];          // skip input h, read then overwritten in place
                out[off] = fmaxf(v, 0.0f);
            }
        }
    }
}

template <int F, int NBOARD>
__global__ __launch_bounds__(256, 1) void k_resnet_fwd(const float* __restrict__ x, int n_boards,
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

    // zero both activation buffers' halos and the stem input (interior rewritten below)
    for (int i = tid; i < 2 * NBOARD * 100; i += 256) {
        const int px = i % 100, r = px / 10, c = px % 10;
        if (r == 0 || r == 9 || c == 0 || c == 9) {
            float* dst = smem + (size_t)(i / 100) * 100 * C::CS + (size_t)px * C::CS;
            for (int k = 0; k < F; k += 4) *reinterpret_cast<float4*>(dst + k) = make_float4(0, 0, 0, 0);
        }
    }
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
            actA[(b * 100 + (r + 1) * 10 + c + 1) * C::CS + n] = fmaxf(acc + bn, 0.0f);
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
        const float* a = actA + (b * 100 + (px / 8 + 1) * 10 + px % 8 + 1) * C::CS;
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
