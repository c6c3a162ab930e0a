// rvz_resnet_alt.hip — the leaf evaluator's A/B alternatives and parity cross-checks, built into
// tools/alt/librvz_alt.so (NOT the product librvz.so; tools/alt/alt_eval.py binds them):
//
//  * k_resnet_fwd (rvz_resnet_fwd_f32): the f32-input MFMA v_mfma_f32_32x32x2_f32 — bit-for-bit
//    k-ordered fp32 FMA chains, the reference's precision, at the f32 matrix rate (157 TF/s).
//  * k_resnet_split (rvz_resnet_fwd_split): every fp32 operand split exactly into three bf16
//    parts, x = x0 + (x1 + x2) (8 significant bits each, 24 together), and the conv GEMMs run on
//    v_mfma_f32_16x16x32_bf16 with the six partial products whose weight is >= 2^-16:
//    x0w0 into one fp32 accumulator, x0w1 + x1w0 + x1w1 + x0w2 + x2w0 into a second.
//    The dropped terms (x1w2, x2w1, x2w2) are <= ~2^-24 of |x w|, i.e. below one fp32 rounding of
//    the product, so the error matches an fp32 GEMM's. The product's h2 kernel (2 f16 parts,
//    3 products) replaced it: half the MFMAs.
//  * k_heads_fc: the FC heads on the VALU (k_heads_mfma's predecessor).
//
// f32 kernel layout (one workgroup = 4 waves = NBOARD boards; F filters; 8x8 boards):
//   LDS act[2][NBOARD][64 pixels][F + 4 floats]   (ping-pong h / y; no halo: taps that leave the
//   board are masked to 0). A pixel row is F + 4 floats, so consecutive pixels start 4 banks apart.
//   conv layer = GEMM  M = NBOARD*64 pixels, N = F, K = 9 taps x F channels, on
//   v_mfma_f32_32x32x2_f32: A lane l = (pixel l&31 of a 32-pixel M-tile, k-slot l>>5), B lane l =
//   (k-slot l>>5, channel l&31 of the N-tile); k-slot h of step s is input channel h*(F/2)+s, so
//   one ds_read_b128 (A) / global_load_dwordx4 (B) feeds 4 steps.
//   Wave w: N-tile, 2 M-tiles -> 2 accumulators of 16 floats.
#include "../../alphazero-reversi_amd/csrc/rvz_resnet_common.hip.h"
#include "rvz_alt.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// ---------------------------------------------------------------------------------------------
// exact 3-part bf16 split of an fp32 value

__device__ __forceinline__ uint32_t bf16_rne(float x) {      // finite x
    const uint32_t u = __float_as_uint(x);
    return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}
__device__ __forceinline__ float bf16_f(uint32_t h) { return __uint_as_float(h << 16); }

// x == h0 + (h1 + h2) exactly: x - h0 is exact (Sterbenz), carries <= 16 significant bits, and
// its remainder after rounding to 8 bits carries <= 8, so h2 is exact too.
__device__ __forceinline__ void split3(float x, uint16_t& h0, uint16_t& h1, uint16_t& h2) {
    const uint32_t b0 = bf16_rne(x);
    const float r1 = x - bf16_f(b0);
    const uint32_t b1 = bf16_rne(r1);
    const float r2 = r1 - bf16_f(b1);
    h0 = (uint16_t)b0;
    h1 = (uint16_t)b1;
    h2 = (uint16_t)bf16_rne(r2);
}
__device__ __forceinline__ float join3(uint16_t h0, uint16_t h1, uint16_t h2) {
    return bf16_f(h0) + (bf16_f(h1) + bf16_f(h2));
}

// the same split for two values with v_cvt_pk_bf16_f32 (round to nearest even, as bf16_rne)
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 bf16x2_f(uint32_t h) {
    return f32x2{__uint_as_float(h << 16), __uint_as_float(h & 0xFFFF0000u)};
}
__device__ __forceinline__ uint32_t cvt2(f32x2 x) {
    const bf16x2 b = __builtin_convertvector(x, bf16x2);
    return __builtin_bit_cast(uint32_t, b);
}
__device__ __forceinline__ void split3x2(f32x2 x, uint32_t& h0, uint32_t& h1, uint32_t& h2) {
    h0 = cvt2(x);
    const f32x2 r1 = x - bf16x2_f(h0);
    h1 = cvt2(r1);
    h2 = cvt2(r1 - bf16x2_f(h1));
}

// ---------------------------------------------------------------------------------------------
// activation accessors: the stem writes, the heads read, through these

struct ActF32 {
    float* p;
    int cs;
    __device__ void store(int row, int n, float v) const { p[row * cs + n] = v; }
    __device__ float load(int row, int k) const { return p[row * cs + k]; }
    __device__ float mul(int) const { return 1.0f; }   // head_convs' per-board scale: none
    __device__ void load8(int row, int k0, float (&v)[8]) const {
        const f32x4 a = *reinterpret_cast<const f32x4*>(p + row * cs + k0);
        const f32x4 b = *reinterpret_cast<const f32x4*>(p + row * cs + k0 + 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) { v[j] = a[j]; v[4 + j] = b[j]; }
    }
};

struct ActSplit {
    uint16_t* p;
    int cs, plane;
    __device__ void store(int row, int n, float v) const {
        uint16_t a, b, c;
        split3(v, a, b, c);
        uint16_t* o = p + row * cs + n;
        o[0] = a;
        o[plane] = b;
        o[2 * plane] = c;
    }
    __device__ float load(int row, int k) const {
        const uint16_t* o = p + row * cs + k;
        return join3(o[0], o[plane], o[2 * plane]);
    }
    __device__ float mul(int) const { return 1.0f; }   // head_convs' per-board scale: none
    __device__ void load8(int row, int k0, float (&v)[8]) const {
        typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));
        const uint16_t* o = p + row * cs + k0;
        const u16x8 a = *reinterpret_cast<const u16x8*>(o);
        const u16x8 b = *reinterpret_cast<const u16x8*>(o + plane);
        const u16x8 c = *reinterpret_cast<const u16x8*>(o + 2 * plane);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = join3(a[j], b[j], c[j]);
    }
};

// leaf planes x[g][3][BS][BS] -> xin[b][10x10 padded pixel][4] (halo and, for BS < 8, the
// unused rows/columns 0)
template <int NBOARD, int BS = 8>
__device__ __forceinline__ void load_input(const float* __restrict__ x, int n_boards, int g0,
                                           float* xin, int tid, int nthr) {
    constexpr int CELLS = BS * BS;
    for (int i = tid; i < NBOARD * 100 * 4; i += nthr) xin[i] = 0.0f;
    __syncthreads();
    for (int i = tid; i < NBOARD * 3 * CELLS; i += nthr) {
        const int b = i / (3 * CELLS), rem = i % (3 * CELLS), ch = rem / CELLS,
                  cell = rem % CELLS;
        const int g = g0 + b;
        const float v = g < n_boards ? x[(size_t)g * 3 * CELLS + rem] : 0.0f;
        xin[(b * 100 + (cell / BS + 1) * 10 + (cell % BS) + 1) * 4 + ch] = v;
    }
}

// stem: conv 3 -> F (VALU; 0.4% of the FLOPs), bias, ReLU -> act rows b*64 + px.
// Lane = pixel (the 27 input taps read from LDS once), wave = (board, group of channels) with the
// group's weights wave-uniform (scalar loads).
template <int F, int NBOARD, int NTHR, class Act>
__device__ __forceinline__ void stem(const float* xin, const Act& act, const float* __restrict__ prm,
                                     const Layout& L, int tid) {
    constexpr int NW = NTHR / 64, CG = NW / NBOARD, CPG = F / CG;
    static_assert(NW % NBOARD == 0 && F % CG == 0, "wave -> (board, channel group)");
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), px = tid & 63;
    const int b = wave % NBOARD, cg = wave / NBOARD, r = px >> 3, c = px & 7;
    float in[27];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int ch = 0; ch < 3; ++ch)
            in[t * 3 + ch] = xin[(b * 100 + (r + t / 3) * 10 + (c + t % 3)) * 4 + ch];
    const float* w = prm + L.stem_w + (int64_t)cg * CPG * 27;
    const float* bias = prm + L.stem_b + cg * CPG;
#pragma unroll 4
    for (int j = 0; j < CPG; ++j) {
        float acc = 0.0f;
#pragma unroll
        for (int k = 0; k < 27; ++k) acc = fmaf(in[k], w[j * 27 + k], acc);
        act.store(b * 64 + px, cg * CPG + j, fmaxf(acc + bias[j], 0.0f));
    }
}

// heads, part 2 (in-kernel form): policy fc (2 cells -> cells + 1), value fc1 (cells -> 256,
// ReLU), value fc2 (256 -> 1) + tanh, for the NBOARD boards of a workgroup; hpv in LDS (rows of
// 192: policy planes, then the value plane)
template <int NBOARD, int NTHR, int BS = 8>
__device__ __forceinline__ void head_fcs(const float* hpv, float* h1,
                                         const float* __restrict__ prm, const Layout& L, int g0,
                                         int n_boards, float* __restrict__ logits,
                                         float* __restrict__ value, int tid) {
    constexpr int CELLS = BS * BS, POUT = CELLS + 1, PIN = 2 * CELLS, ROWS = POUT + 256;
    const int lane = tid & 63;
    // thread per output row, f32x4 loads
    for (int o = tid; o < NBOARD * ROWS; o += NTHR) {
        const int b = o / ROWS, rem = o % ROWS;
        const int g = g0 + b;
        if (rem < POUT) {
            const f32x4* wr = reinterpret_cast<const f32x4*>(prm + L.pfc_w + rem * PIN);
            const f32x4* in = reinterpret_cast<const f32x4*>(hpv + b * 192);
            float acc = prm[L.pfc_b + rem];
#pragma unroll 16
            for (int i = 0; i < PIN / 4; ++i) {
                const f32x4 w = wr[i], v = in[i];
                acc = fmaf(v[0], w[0], acc);
                acc = fmaf(v[1], w[1], acc);
                acc = fmaf(v[2], w[2], acc);
                acc = fmaf(v[3], w[3], acc);
            }
            if (g < n_boards) logits[(size_t)g * POUT + rem] = acc;
        } else {
            const int u = rem - POUT;
            const f32x4* wr = reinterpret_cast<const f32x4*>(prm + L.vfc1_w + u * CELLS);
            const f32x4* in = reinterpret_cast<const f32x4*>(hpv + b * 192 + PIN);
            float acc = prm[L.vfc1_b + u];
#pragma unroll
            for (int i = 0; i < CELLS / 4; ++i) {
                const f32x4 w = wr[i], v = in[i];
                acc = fmaf(v[0], w[0], acc);
                acc = fmaf(v[1], w[1], acc);
                acc = fmaf(v[2], w[2], acc);
                acc = fmaf(v[3], w[3], acc);
            }
            h1[b * 256 + u] = fmaxf(acc, 0.0f);
        }
    }
    __syncthreads();
    // value fc2 (256 -> 1) + tanh: one wave per board
    const int wave = tid >> 6;
    for (int b = wave; b < NBOARD; b += NTHR / 64) {
        float acc = 0.0f;
        for (int i = lane; i < 256; i += 64) acc = fmaf(h1[b * 256 + i], prm[L.vfc2_w + i], acc);
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
        const int g = g0 + b;
        if (lane == 0 && g < n_boards) value[g] = tanhf(acc + prm[L.vfc2_b]);
    }
}

// heads, part 2 as its own launch over FCB boards per workgroup (the split path): each FC weight
// row is loaded once per workgroup into registers and applied to all FCB boards (LDS broadcast
// inputs) — inside the trunk kernel the same weights streamed from L2 once per 2 boards, with
// the matrix cores idle. Thread t: value-fc1 row t; threads < 2*(cells+1): half of policy row
// t/2. work rows: [2 cells policy planes | cells value plane], stride 192.
#ifndef RVZ_FCB
#define RVZ_FCB 8
#endif
constexpr int FCB = RVZ_FCB;   // boards per workgroup (multiple of 4)
static_assert(RVZ_LIVE_STRIPE % FCB == 0 && RVZ_LIVE_STRIPE % 16 == 0, "stripe granules");

template <int BS>
__global__ __launch_bounds__(256) void k_heads_fc(const float* __restrict__ work, int n,
                                                  const float* __restrict__ prm, Layout L,
                                                  float* __restrict__ logits,
                                                  float* __restrict__ value,
                                                  const int32_t* __restrict__ n_live,
                                                  uint32_t* __restrict__ stamp_ctr) {
    // bench.py: the trunk launch before this one is complete; advance its stamp ring
    if (stamp_ctr && blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(stamp_ctr, 1u);
    if (row_dead(n_live, (int)blockIdx.x * FCB)) return;   // the workgroup's rows are all dead
    constexpr int CELLS = BS * BS, PIN = 2 * CELLS, POUT = CELLS + 1, ROW = 3 * CELLS;
    constexpr int VQ = CELLS / 4, PQ = PIN / 2 / 4;   // f32x4 per value row / policy half-row
    static_assert(CELLS % 4 == 0 && 2 * POUT <= 256, "thread map");
    __shared__ __attribute__((aligned(16))) float in[FCB][ROW];
    __shared__ __attribute__((aligned(16))) float h1[FCB][256];
    __shared__ float pp[FCB][2 * POUT];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g0 = blockIdx.x * FCB, nb = n - g0 < FCB ? n - g0 : FCB;
    f32x4 wv[VQ], wp[PQ];
    {
        const f32x4* r = reinterpret_cast<const f32x4*>(prm + L.vfc1_w + tid * CELLS);
#pragma unroll
        for (int i = 0; i < VQ; ++i) wv[i] = r[i];
    }
    if (tid < 2 * POUT) {
        const f32x4* r = reinterpret_cast<const f32x4*>(prm + L.pfc_w + (tid >> 1) * PIN +
                                                         (tid & 1) * (PIN / 2));
#pragma unroll
        for (int i = 0; i < PQ; ++i) wp[i] = r[i];
    }
    for (int i = tid; i < FCB * ROW; i += 256) {
        const int b = i / ROW, k = i % ROW;
        (&in[0][0])[i] = b < nb ? work[(size_t)(g0 + b) * 192 + k] : 0.0f;
    }
    __syncthreads();
    // 4 boards at a time: four independent FMA chains per thread
    constexpr int IL = 4;
    const float b1 = prm[L.vfc1_b + tid];
    for (int b0 = 0; b0 < FCB; b0 += IL) {
        float acc[IL];
#pragma unroll
        for (int j = 0; j < IL; ++j) acc[j] = b1;
#pragma unroll
        for (int i = 0; i < VQ; ++i)
#pragma unroll
            for (int j = 0; j < IL; ++j) {
                const f32x4 x = reinterpret_cast<const f32x4*>(&in[b0 + j][PIN])[i];
                acc[j] = fmaf(x[0], wv[i][0], acc[j]);
                acc[j] = fmaf(x[1], wv[i][1], acc[j]);
                acc[j] = fmaf(x[2], wv[i][2], acc[j]);
                acc[j] = fmaf(x[3], wv[i][3], acc[j]);
            }
#pragma unroll
        for (int j = 0; j < IL; ++j) h1[b0 + j][tid] = fmaxf(acc[j], 0.0f);
    }
    if (tid < 2 * POUT) {
        for (int b0 = 0; b0 < FCB; b0 += IL) {
            float acc[IL] = {};
#pragma unroll
            for (int i = 0; i < PQ; ++i)
#pragma unroll
                for (int j = 0; j < IL; ++j) {
                    const f32x4 x =
                        reinterpret_cast<const f32x4*>(&in[b0 + j][(tid & 1) * (PIN / 2)])[i];
                    acc[j] = fmaf(x[0], wp[i][0], acc[j]);
                    acc[j] = fmaf(x[1], wp[i][1], acc[j]);
                    acc[j] = fmaf(x[2], wp[i][2], acc[j]);
                    acc[j] = fmaf(x[3], wp[i][3], acc[j]);
                }
#pragma unroll
            for (int j = 0; j < IL; ++j) pp[b0 + j][tid] = acc[j];
        }
    }
    __syncthreads();
    for (int o = tid; o < nb * POUT; o += 256) {
        const int b = o / POUT, r = o % POUT;
        logits[(size_t)(g0 + b) * POUT + r] =
            prm[L.pfc_b + r] + (pp[b][2 * r] + pp[b][2 * r + 1]);
    }
    for (int b = wave; b < nb; b += 4) {
        float acc = 0.0f;
        for (int i = lane; i < 256; i += 64) acc = fmaf(h1[b][i], prm[L.vfc2_w + i], acc);
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
        if (lane == 0) value[g0 + b] = tanhf(acc + prm[L.vfc2_b]);
    }
}

// =============================================================================================
// f32 MFMA kernel

template <int F, int NBOARD>
struct Cfg {
    static constexpr int CS = F + 4;                 // padded channel stride (bank spread)
    static constexpr int BOARD = 64 * CS;            // floats per board per buffer
    static constexpr int ACT = NBOARD * BOARD;       // floats per buffer
    static constexpr int XIN = NBOARD * 100 * 4;     // stem input, 3 planes padded to 4 (halo)
    static constexpr int HPV = NBOARD * 192;         // 1x1 conv outputs (policy NCHW, value)
    static constexpr int H1 = NBOARD * 256;          // value fc1 output
    static constexpr int SMEM = 2 * ACT + XIN + HPV + H1;
    static constexpr int MTILES = 2 * NBOARD;        // 32-pixel M-tiles (4 board rows each)
    static constexpr int NTILES = F / 32;            // 32-channel N-tiles
    static_assert(MTILES * NTILES == 8, "8 tiles = 4 waves x 2 accumulators");
    static_assert(SMEM * 4 <= 160 * 1024, "fits the 160 KiB LDS of a CU");
};

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
    float* hpv = xin + C::XIN;
    float* h1 = hpv + C::HPV;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g0 = blockIdx.x * NBOARD;

    load_input<NBOARD>(x, n_boards, g0, xin, tid, 256);
    __syncthreads();
    stem<F, NBOARD, 256>(xin, ActF32{actA, C::CS}, prm, L, tid);
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
    head_convs<F, NBOARD, 256>(ActF32{actA, C::CS}, actB, prm, L, HeadsLds{hpv}, tid);
    __syncthreads();
    head_fcs<NBOARD, 256>(hpv, h1, prm, L, g0, n_boards, logits, value, tid);
}

// =============================================================================================
// split (3 x bf16) kernel
//
// LDS: act[2 buffers][3 parts][NBOARD*64 + 1 rows][F + 8 bf16]. Row NBOARD*64 stays zero: the
// off-board taps of the 3x3 conv read it (no halo, no select). A row is F + 8 bf16 = an odd
// number S of 16-byte slots. A ds_read_b128 is serviced in the lane groups {0-3,12-15,20-27},
// {4-11,16-19,28-31} (+32 for the other half); here a half-wave reads 32 consecutive pixels at
// one k-offset, so each group holds 16 pixels covering all residues mod 16 and slot(px) =
// S*px mod 16 is distinct inside the group: conflict-free.
// GEMM per conv layer, computed transposed (D = W X^T) on v_mfma_f32_32x32x16_bf16: M = F output
// channels (32-channel tiles), N = NBOARD*64 pixels (32-pixel tiles), K = 9 taps x F (16-channel
// k-steps). 8 waves, one 32x32 output tile each (F=64: 2 channel x 4 pixel tiles over 2 boards;
// F=128: 4 x 2 over 1 board); per k-step a wave reads 3 activation fragments (LDS), loads 3
// weight fragments (L2, prefetched two k-steps ahead) and issues 6 MFMAs (192 cycles), which
// leaves most of each MFMA's issue gap free for the loads.
// Lane maps: A lane l = out-channel l&31, in-channels 8(l>>5)..+7 (weights); B lane l = pixel
// l&31, in-channels 8(l>>5)..+7 (activations); D col = l&31 = pixel, row = (reg&3) + 8(reg>>2) +
// 4(l>>5) = out-channel: a lane ends with 4 runs of 4 consecutive channels of one pixel, stored
// with 8-byte writes.
// Split weights (rvz_resnet_split_weights): frag[layer][tap][kstep][part][ctile][lane][8] bf16,
// so one wave's fragment is 1 KiB contiguous (one coalesced global_load_dwordx4 per lane).



// MFMA shape traits (D = W X^T: TM output channels x TN pixels, K input channels per step)
struct Shape32 {   // v_mfma_f32_32x32x16_bf16 (RVZ_SPLIT_SHAPE=32)
    [[maybe_unused]] static constexpr int TM = 32, TN = 32, K = 16, NG = 4;
    typedef f32x16 acc_t;
    // channel offset (within the tile) of register group g; registers 4g .. 4g+3
    static __device__ __forceinline__ int chan(int g, int lane) { return 8 * g + 4 * (lane >> 5); }
    static __device__ __forceinline__ acc_t mfma(bf16x8 a, bf16x8 b, acc_t c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
    }
};
struct Shape16 {   // v_mfma_f32_16x16x32_bf16
    static constexpr int TM = 16, TN = 16, K = 32, NG = 1;
    typedef f32x4 acc_t;
    static __device__ __forceinline__ int chan(int, int lane) { return 4 * (lane >> 4); }
    static __device__ __forceinline__ acc_t mfma(bf16x8 a, bf16x8 b, acc_t c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    }
};

// 16x16x32 by default: on random data the chip holds a higher clock on it than on 32x32x16
// (MI355X_MICROARCH.md 'DVFS give-back' item 7); measured 0.875 vs 0.942 ms per C2 leaf batch
#ifndef RVZ_SPLIT_SHAPE
#define RVZ_SPLIT_SHAPE 16
#endif
#if RVZ_SPLIT_SHAPE == 16
typedef Shape16 SplitShape;
#ifndef RVZ_SPLIT_CTW
#define RVZ_SPLIT_CTW 2      // channel tiles per wave
#define RVZ_SPLIT_PTW 4      // pixel tiles per wave
#endif
#else
typedef Shape32 SplitShape;
#ifndef RVZ_SPLIT_CTW
#define RVZ_SPLIT_CTW 1
#define RVZ_SPLIT_PTW 2
#endif
#endif

template <class S, int F, int NBOARD>
struct CfgS {
    // a row is F + PAD bf16 = R 16-byte slots. ds_read_b128 lane groups are {0-3,12-15,20-27},
    // {4-11,16-19,28-31} (+32). 32x32x16: a half-wave reads 32 consecutive pixels at one
    // k-offset, every group holds all 16 pixel residues mod 16 -> R odd is conflict-free.
    // 16x16x32: a group holds pixels {0-3,12-15} at k-offset q and {4-11} at q+1 -> R = 2 mod 4.
    static constexpr int CSB = S::TM == 32 ? F + 8 : F + 16;   // bf16 per pixel row
    static constexpr int ZROW = NBOARD * 64;         // the zero row
    static constexpr int PLANE = (ZROW + 1) * CSB;   // bf16 per part
    static constexpr int ACT = 3 * PLANE;            // bf16 per buffer
    static constexpr int XIN = NBOARD * 100 * 4;     // floats
    static constexpr int BYTES = 2 * ACT * 2 + 4 * XIN;
    static constexpr int KS = F / S::K;              // k-steps per tap
    static constexpr int NIT = 9 * KS;               // k-steps per layer
    static constexpr int CT = F / S::TM;             // channel tiles
    static_assert(S::TM == 32 ? (CSB * 2 / 16) % 2 == 1 : (CSB * 2 / 16) % 4 == 2,
                  "conflict-free row stride");
    static_assert((PLANE * 2) % 16 == 0, "16-byte aligned parts");
    static_assert(BYTES <= 160 * 1024, "fits the 160 KiB LDS of a CU");
};

#ifndef RVZ_SPLIT_PD
#define RVZ_SPLIT_PD 3       // weight prefetch distance, k-steps
#endif
#ifndef RVZ_SPLIT_INTERLEAVE
#define RVZ_SPLIT_INTERLEAVE 1   // loads placed between the MFMAs of a k-step
#endif
#define RVZ_SPLIT_PAD 4      // k-steps of padding after the last layer's weights (>= PD)
static_assert(RVZ_SPLIT_PD <= RVZ_SPLIT_PAD, "prefetch stays inside the padded buffer");

__host__ __device__ inline int64_t split_layer_elems(int F) { return (int64_t)9 * F * F * 3; }
__host__ __device__ inline int64_t split_kstep_elems(int F) {   // one k-step, all parts/tiles
    return (int64_t)3 * F * SplitShape::K;
}

// the wave's tiles: CTW channel tiles x PTW pixel tiles
template <class S, int F, int CTW, int PTW>
struct WaveTiles {
    static constexpr int CG = F / (CTW * S::TM);     // channel groups (waves along channels)
    int ct0, px[PTW];
    __device__ WaveTiles(int wave, int lane) {
        ct0 = (wave % CG) * CTW;
        const int pt0 = (wave / CG) * PTW;
#pragma unroll
        for (int u = 0; u < PTW; ++u) px[u] = (pt0 + u) * S::TN + lane % S::TN;
    }
};

// conv epilogue: bias (+ skip), ReLU, exact split back into the three parts; per register group
// g of tile (c, u) the lane holds 4 consecutive channels of its pixel -> 8-byte writes. The skip
// input of a residual block is the block input, which this lane itself produced (same tile map
// in the stem and every conv): it stays in registers (res, fp32 — the exact value its split
// encodes), RES adds it, KEEP stores the result as the next block's skip input.
template <class S, int CTW, int PTW, bool REGRES>
struct EpiRegs {
    f32x4 bias[CTW][S::NG];
    float res[CTW][PTW][REGRES ? S::NG * 4 : 1];
};
// skip input in registers where they fit (F = 64); at F = 128 they would spill, and the epilogue
// re-reads it from LDS (joining its split)
template <int F>
struct RegRes {
    static constexpr bool value = F <= 64;
};

template <class S, int F, int NBOARD, int CTW, int PTW, bool RES, bool KEEP>
__device__ __forceinline__ void epilogue_split(uint16_t* __restrict__ out,
                                               const typename S::acc_t (&hi)[CTW][PTW],
                                               const typename S::acc_t (&lo)[CTW][PTW],
                                               EpiRegs<S, CTW, PTW, RegRes<F>::value>& er,
                                               const WaveTiles<S, F, CTW, PTW>& wt, int lane) {
    using C = CfgS<S, F, NBOARD>;
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int c = 0; c < CTW; ++c)
#pragma unroll
        for (int u = 0; u < PTW; ++u)
#pragma unroll
            for (int g = 0; g < S::NG; ++g) {
                const int n0 = (wt.ct0 + c) * S::TM + S::chan(g, lane);
                uint16_t* o = out + wt.px[u] * C::CSB + n0;
                constexpr bool REG = RegRes<F>::value;
                typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));
                u16x4 s0, s1, s2;
                if (RES && !REG) {
                    s0 = *reinterpret_cast<const u16x4*>(o);
                    s1 = *reinterpret_cast<const u16x4*>(o + C::PLANE);
                    s2 = *reinterpret_cast<const u16x4*>(o + 2 * C::PLANE);
                }
                u32x2 d0, d1, d2;
#pragma unroll
                for (int hf = 0; hf < 2; ++hf) {
                    f32x2 v;
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        const int j = 2 * hf + e, reg = 4 * g + j;
                        v[e] = (hi[c][u][reg] + lo[c][u][reg]) + er.bias[c][g][j];
                        if (RES) {                              // skip input
                            if constexpr (REG) v[e] += er.res[c][u][reg];
                            else v[e] += join3(s0[j], s1[j], s2[j]);
                        }
                        v[e] = fmaxf(v[e], 0.0f);
                        if constexpr (KEEP && REG) er.res[c][u][reg] = v[e];
                    }
                    uint32_t h0, h1, h2;
                    split3x2(v, h0, h1, h2);
                    d0[hf] = h0;
                    d1[hf] = h1;
                    d2[hf] = h2;
                }
                *reinterpret_cast<u32x2*>(o) = d0;
                *reinterpret_cast<u32x2*>(o + C::PLANE) = d1;
                *reinterpret_cast<u32x2*>(o + 2 * C::PLANE) = d2;
            }
}

template <class S, int F, int CTW, int PTW>
__device__ __forceinline__ void load_bias(EpiRegs<S, CTW, PTW, RegRes<F>::value>& er, const float* __restrict__ bias,
                                          const WaveTiles<S, F, CTW, PTW>& wt, int lane) {
#pragma unroll
    for (int c = 0; c < CTW; ++c)
#pragma unroll
        for (int g = 0; g < S::NG; ++g)
            er.bias[c][g] = *reinterpret_cast<const f32x4*>(bias + (wt.ct0 + c) * S::TM +
                                                            S::chan(g, lane));
}

// 8 bf16 parts p of 8 fp32 values
__device__ __forceinline__ void split8(const float (&v)[8], bf16x8 (&out)[3]) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    u32x4 w0, w1, w2;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        uint32_t a, b, c;
        split3x2(f32x2{v[2 * i], v[2 * i + 1]}, a, b, c);
        w0[i] = a;
        w1[i] = b;
        w2[i] = c;
    }
    out[0] = __builtin_bit_cast(bf16x8, w0);
    out[1] = __builtin_bit_cast(bf16x8, w1);
    out[2] = __builtin_bit_cast(bf16x8, w2);
}

// the six partial products: (weight part, activation part), hi first
__device__ constexpr int kTW[6] = {0, 0, 2, 1, 0, 1};
__device__ constexpr int kTA[6] = {0, 2, 0, 1, 1, 0};

// stem conv 3 -> F (network.py:33-34 + BN folded) as a K = 27 (padded to 32) GEMM on the same
// split MFMA and tile map as the trunk: k = tap*3 + ch; A = stem weights (split in registers),
// B = the input taps read from the halo-padded xin; epilogue into actA.
template <class S, int F, int NBOARD, int CTW, int PTW>
__device__ __forceinline__ void stem_split(const float* xin, uint16_t* __restrict__ out,
                                           const float* __restrict__ prm, const Layout& L,
                                           int wave, int lane,
                                           EpiRegs<S, CTW, PTW, RegRes<F>::value>& er) {
    const WaveTiles<S, F, CTW, PTW> wt(wave, lane);
    load_bias(er, prm + L.stem_b, wt, lane);
    const int kq = 8 * (lane / S::TM);               // this lane's k offset in a step
    typename S::acc_t hi[CTW][PTW], lo[CTW][PTW];
#pragma unroll
    for (int c = 0; c < CTW; ++c)
#pragma unroll
        for (int u = 0; u < PTW; ++u) {
            hi[c][u] = typename S::acc_t{};
            lo[c][u] = typename S::acc_t{};
        }
#pragma unroll
    for (int ks = 0; ks < 32 / S::K; ++ks) {
        bf16x8 wq[CTW][3], aq[PTW][3];
#pragma unroll
        for (int c = 0; c < CTW; ++c) {
            const float* wrow = prm + L.stem_w + ((wt.ct0 + c) * S::TM + lane % S::TM) * 27;
            float wv[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int k = ks * S::K + kq + j;
                wv[j] = k < 27 ? wrow[k] : 0.0f;
            }
            split8(wv, wq[c]);
        }
#pragma unroll
        for (int u = 0; u < PTW; ++u) {
            const int px = wt.px[u], b = px >> 6, r = (px & 63) >> 3, cc = px & 7;
            float xv[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int k = ks * S::K + kq + j, t = k / 3, ch = k % 3;
                xv[j] = k < 27 ? xin[(b * 100 + (r + t / 3) * 10 + (cc + t % 3)) * 4 + ch] : 0.0f;
            }
            split8(xv, aq[u]);
        }
#pragma unroll
        for (int term = 0; term < 6; ++term)
#pragma unroll
            for (int c = 0; c < CTW; ++c)
#pragma unroll
                for (int u = 0; u < PTW; ++u) {
                    auto& acc = term == 0 ? hi[c][u] : lo[c][u];
                    acc = S::mfma(wq[c][kTW[term]], aq[u][kTA[term]], acc);
                }
    }
    epilogue_split<S, F, NBOARD, CTW, PTW, false, true>(out, hi, lo, er, wt, lane);
}


template <class S, int F, int NBOARD, int CTW, int PTW, bool RES, int BS = 8>
__device__ __forceinline__ void conv_split(const uint16_t* __restrict__ in,
                                           uint16_t* __restrict__ out,
                                           const uint16_t* __restrict__ wl,   // layer fragments
                                           const float* __restrict__ bias, int wave, int lane,
                                           bf16x8 (&bc)[RVZ_SPLIT_PD][CTW][3],
                                           EpiRegs<S, CTW, PTW, RegRes<F>::value>& er,
                                           int ptag = -1) {
    using C = CfgS<S, F, NBOARD>;
    constexpr int KS = C::KS, CT = C::CT, NIT = C::NIT, PD = RVZ_SPLIT_PD;
    const WaveTiles<S, F, CTW, PTW> wt(wave, lane);
    load_bias(er, bias, wt, lane);                  // lands during the k-loop
    const int kq = 8 * (lane / S::TM);
    // the taps of each of the lane's pixels that stay on its board
    unsigned pmask[PTW];
#pragma unroll
    for (int u = 0; u < PTW; ++u) {
        const int rr = (wt.px[u] & 63) >> 3, cc = wt.px[u] & 7;
        unsigned msk = 0;
#pragma unroll
        for (int t = 0; t < 9; ++t)
            if ((unsigned)(rr + t / 3 - 1) < (unsigned)BS && (unsigned)(cc + t % 3 - 1) < (unsigned)BS)
                msk |= 1u << t;
        pmask[u] = msk;
    }
    typename S::acc_t hi[CTW][PTW], lo[CTW][PTW];
#pragma unroll
    for (int c = 0; c < CTW; ++c)
#pragma unroll
        for (int u = 0; u < PTW; ++u) {
            hi[c][u] = typename S::acc_t{};
            lo[c][u] = typename S::acc_t{};
        }
    // fragment (it, part, ctile) of this lane: wf[((it*3 + part)*CT + ctile)*64]
    const bf16x8* wf = reinterpret_cast<const bf16x8*>(wl) + wt.ct0 * 64 + lane;
    auto load_b = [&](bf16x8 (&bq)[CTW][3], int it) {
#pragma unroll
        for (int c = 0; c < CTW; ++c)
#pragma unroll
            for (int p = 0; p < 3; ++p) bq[c][p] = wf[((it * 3 + p) * CT + c) * 64];
    };
    auto load_a = [&](bf16x8 (&aq)[PTW][3], int it) {
        const int t = it / KS, ks = it - t * KS;
        const int off = (t / 3 - 1) * 8 + (t % 3 - 1);
#pragma unroll
        for (int u = 0; u < PTW; ++u) {
            const int row = (pmask[u] >> t) & 1u ? wt.px[u] + off : C::ZROW;
            const uint16_t* ap = in + row * C::CSB + ks * S::K + kq;
#pragma unroll
            for (int p = 0; p < 3; ++p)
                aq[u][p] = *reinterpret_cast<const bf16x8*>(ap + p * C::PLANE);
        }
    };
    // consecutive MFMAs of one wave go to different accumulators
    auto compute = [&](const bf16x8 (&aq)[PTW][3], const bf16x8 (&bq)[CTW][3]) {
#pragma unroll
        for (int term = 0; term < 6; ++term)
#pragma unroll
            for (int c = 0; c < CTW; ++c)
#pragma unroll
                for (int u = 0; u < PTW; ++u) {
                    auto& acc = term == 0 ? hi[c][u] : lo[c][u];
                    acc = S::mfma(bq[c][kTW[term]], aq[u][kTA[term]], acc);
                }
    };
    // Software pipeline, fully unrolled (constant register indices, no copies of in-flight
    // loads): step it computes while step it+APD's activation fragments (LDS) and step it+PD's
    // weight fragments (L2) load, one load per MFMA issue gap (an MFMA leaves most of its issue
    // cycles free; 9+ loads back to back would let the matrix pipe drain). bc carries the next
    // layer's first PD k-steps (layers are contiguous; the buffer has RVZ_SPLIT_PAD k-steps of
    // padding after the last).
    // activation prefetch distance: 2 k-steps where the registers allow (F = 64), else 1
    constexpr int APD = F <= 64 ? 2 : 1;
    bf16x8 bq[NIT + PD][CTW][3];
    bf16x8 aq[APD + 1][PTW][3];
#pragma unroll
    for (int d = 0; d < PD; ++d)
#pragma unroll
        for (int c = 0; c < CTW; ++c)
#pragma unroll
            for (int p = 0; p < 3; ++p) bq[d][c][p] = bc[d][c][p];
#pragma unroll
    for (int d = 0; d < APD; ++d) load_a(aq[d], d);
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
        if (it + APD < NIT) load_a(aq[(it + APD) % (APD + 1)], it + APD);
        load_b(bq[it + PD], it + PD);
#if RVZ_SPLIT_INTERLEAVE
        compute(aq[it % (APD + 1)], bq[it]);
        interleave_loads<0, 6 * CTW * PTW, 3 * PTW, 3 * CTW>();
        __builtin_amdgcn_sched_barrier(0);
#else
        __builtin_amdgcn_sched_barrier(0);
        compute(aq[it % (APD + 1)], bq[it]);
        __builtin_amdgcn_sched_barrier(0);
#endif
    }
#pragma unroll
    for (int d = 0; d < PD; ++d)
#pragma unroll
        for (int c = 0; c < CTW; ++c)
#pragma unroll
            for (int p = 0; p < 3; ++p) bc[d][c][p] = bq[NIT + d][c][p];
    if (ptag >= 0) {
        PHASE(ptag);
        WAVE_T(0);
    }
    // conv A (block input -> t): the skip input stays in er.res; conv B adds it and keeps
    epilogue_split<S, F, NBOARD, CTW, PTW, RES, RES>(out, hi, lo, er, wt, lane);
}

// one workgroup = 4 waves (one per SIMD) = NBOARD boards; wave tile CTW x PTW MFMA tiles
template <class S, int F, int NBOARD, int CTW, int PTW, int BS>
__global__ __launch_bounds__(256, 1) void k_resnet_split(const float* __restrict__ x,
                                                         int n_boards,
                                                         const float* __restrict__ prm, Layout L,
                                                         const uint16_t* __restrict__ wsp,
                                                         int n_blocks, float* __restrict__ work) {
    using C = CfgS<S, F, NBOARD>;
    using WT = WaveTiles<S, F, CTW, PTW>;
    static_assert(WT::CG * (NBOARD * 64 / (PTW * S::TN)) == 4, "4 waves");
    constexpr int NTHR = 256;
    __shared__ __attribute__((aligned(16))) char smem[C::BYTES];
    uint16_t* actA = reinterpret_cast<uint16_t*>(smem);
    uint16_t* actB = actA + C::ACT;
    float* xin = reinterpret_cast<float*>(actB + C::ACT);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g0 = blockIdx.x * NBOARD;
    PHASE(0);
    RT(0);

    // zero rows of both buffers, all parts (6 consecutive planes)
    for (int i = tid; i < 6 * C::CSB; i += NTHR) {
        const int part = i / C::CSB, k = i % C::CSB;
        actA[part * C::PLANE + C::ZROW * C::CSB + k] = 0;
    }
    // the first PD k-steps' weight fragments, in flight during the input and stem
    bf16x8 bc[RVZ_SPLIT_PD][CTW][3];
    if (n_blocks > 0) {
        const bf16x8* wf = reinterpret_cast<const bf16x8*>(wsp) + WT(wave, lane).ct0 * 64 + lane;
#pragma unroll
        for (int s = 0; s < RVZ_SPLIT_PD; ++s)
#pragma unroll
            for (int c = 0; c < CTW; ++c)
#pragma unroll
                for (int p = 0; p < 3; ++p) bc[s][c][p] = wf[((s * 3 + p) * C::CT + c) * 64];
    }
    load_input<NBOARD, BS>(x, n_boards, g0, xin, tid, NTHR);
    __syncthreads();
    const ActSplit outA{actA, C::CSB, C::PLANE};
    EpiRegs<S, CTW, PTW, RegRes<F>::value> er;      // bias and skip-input registers
    stem_split<S, F, NBOARD, CTW, PTW>(xin, actA, prm, L, wave, lane, er);
    __syncthreads();
    PHASE(1);
    const int64_t LW = split_layer_elems(F);
    for (int blk = 0; blk < n_blocks; ++blk) {
        const int l1 = 2 * blk, l2 = 2 * blk + 1;
        conv_split<S, F, NBOARD, CTW, PTW, false, BS>(actA, actB, wsp + l1 * LW,
                                                  prm + L.res_b + (size_t)l1 * F, wave, lane, bc,
                                                  er, blk == 0 ? 4 : -1);
        if (blk == 0) {
            PHASE(5);
            WAVE_T(1);
        }
        __syncthreads();
        if (blk == 0) PHASE(6);
        conv_split<S, F, NBOARD, CTW, PTW, true, BS>(actB, actA, wsp + l2 * LW,
                                                 prm + L.res_b + (size_t)l2 * F, wave, lane, bc,
                                                 er);
        __syncthreads();
    }
    PHASE(2);
    head_convs<F, NBOARD, NTHR, BS>(outA, reinterpret_cast<float*>(actB), prm, L,
                                    HeadsGlobal{work, g0, n_boards}, tid);
    PHASE(3);
    RT(1);
}

// res_w[l][t][n][k] fp32 -> frag[l][t][ks][part][ctile][lane][8] bf16 parts, for SplitShape:
// lane = ((k % K) / 8) * TM + n % TM (the A-operand lane map)
__global__ void k_split_weights(const float* __restrict__ w, int F, int64_t total,
                                uint16_t* __restrict__ out) {
    constexpr int K = SplitShape::K, TM = SplitShape::TM;
    const int KS = F / K, CT = F / TM;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int k = (int)(i % F), n = (int)((i / F) % F);
        const int64_t lt = i / ((int64_t)F * F);             // layer*9 + tap
        const int ks = k / K, j = k % 8, ct = n / TM;
        const int ln = ((k % K) / 8) * TM + n % TM;
        uint16_t h[3];
        split3(w[i], h[0], h[1], h[2]);
#pragma unroll
        for (int p = 0; p < 3; ++p)
            out[((((lt * KS + ks) * 3 + p) * CT + ct) * 64 + ln) * 8 + j] = h[p];
    }
}

}  // namespace

template <int BS>
static void launch_trunk(const float* x, int32_t n, const float* params, const uint16_t* wsplit,
                         int32_t filters, int32_t blocks, float* work, hipStream_t s) {
    const Layout L = make_layout(filters, blocks, BS);
    if (filters == 64)
        hipLaunchKernelGGL((k_resnet_split<SplitShape, 64, 2, RVZ_SPLIT_CTW, RVZ_SPLIT_PTW, BS>),
                           dim3((n + 1) / 2), dim3(256), 0, s, x, n, params, L, wsplit, blocks,
                           work);
    else
        hipLaunchKernelGGL((k_resnet_split<SplitShape, 128, 1, RVZ_SPLIT_CTW, RVZ_SPLIT_PTW, BS>),
                           dim3(n), dim3(256), 0, s, x, n, params, L, wsplit, blocks, work);
}

extern "C" {

int rvz_resnet_fwd_f32(int32_t board, const float* x, int32_t n, const float* params,
                       int32_t filters, int32_t blocks, float* logits, float* value,
                       void* stream) {
    if (board != 8 || !x || !params || !logits || !value || n < 0 || blocks < 0)
        return RVZ_EINVAL;
    if (((uintptr_t)params & 15) != 0) return RVZ_EINVAL;
    if (n == 0) return RVZ_OK;
    const Layout L = make_layout(filters, blocks);
    hipStream_t s = (hipStream_t)stream;
    if (filters == 64) {
        hipLaunchKernelGGL((k_resnet_fwd<64, 2>), dim3((n + 1) / 2), dim3(256), 0, s, x, n, params,
                           L, blocks, logits, value);
    } else if (filters == 128) {
        hipLaunchKernelGGL((k_resnet_fwd<128, 1>), dim3(n), dim3(256), 0, s, x, n, params, L,
                           blocks, logits, value);
    } else {
        return RVZ_EINVAL;
    }
    return hipGetLastError() == hipSuccess ? RVZ_OK : RVZ_EHIP;
}

int64_t rvz_resnet_split_size(int32_t filters, int32_t blocks) {
    if ((filters != 64 && filters != 128) || blocks < 0) return RVZ_EINVAL;
    // + padding: the last layer's weight prefetch runs up to RVZ_SPLIT_PAD steps past the end
    return (int64_t)2 * blocks * split_layer_elems(filters) +
           RVZ_SPLIT_PAD * split_kstep_elems(filters);
}

int rvz_resnet_split_weights(const float* params, int32_t filters, int32_t blocks, uint16_t* out,
                             void* stream) {
    if (!params || (!out && blocks > 0) || (filters != 64 && filters != 128) || blocks < 0)
        return RVZ_EINVAL;
    if (blocks == 0) return RVZ_OK;
    const Layout L = make_layout(filters, blocks);
    const int64_t total = (int64_t)2 * blocks * 9 * filters * filters;
    const int64_t nblk = (total + 255) / 256;
    hipLaunchKernelGGL(k_split_weights, dim3((unsigned)(nblk < 4096 ? nblk : 4096)), dim3(256), 0,
                       (hipStream_t)stream, params + L.res_w, filters, total, out);
    return hipGetLastError() == hipSuccess ? RVZ_OK : RVZ_EHIP;
}

int rvz_resnet_trunk_split(int32_t board, const float* x, int32_t n, const float* params,
                           const uint16_t* wsplit, int32_t filters, int32_t blocks, float* work,
                           void* stream) {
    if (!x || !params || (!wsplit && blocks > 0) || !work || n < 0 || blocks < 0 ||
        (board != 8 && board != 6) || (filters != 64 && filters != 128))
        return RVZ_EINVAL;
    if (((uintptr_t)params & 15) != 0 || ((uintptr_t)wsplit & 15) != 0) return RVZ_EINVAL;
    if (n == 0) return RVZ_OK;
    hipStream_t s = (hipStream_t)stream;
    if (board == 8) launch_trunk<8>(x, n, params, wsplit, filters, blocks, work, s);
    else launch_trunk<6>(x, n, params, wsplit, filters, blocks, work, s);
    return hipGetLastError() == hipSuccess ? RVZ_OK : RVZ_EHIP;
}

// the FC heads on the VALU (FCB boards per workgroup): k_heads_mfma's predecessor
int rvz_alt_heads_valu(int32_t board, const float* work, int32_t n, const float* params,
                       int32_t filters, int32_t blocks, float* logits, float* value,
                       void* stream) {
    if (!work || !params || !logits || !value || n < 0 || blocks < 0 ||
        (board != 8 && board != 6) || (filters != 64 && filters != 128))
        return RVZ_EINVAL;
    if (n == 0) return RVZ_OK;
    const Layout L = make_layout(filters, blocks, board);
    const dim3 grid((n + FCB - 1) / FCB), block(256);
    if (board == 8)
        hipLaunchKernelGGL(k_heads_fc<8>, grid, block, 0, (hipStream_t)stream, work, n, params,
                           L, logits, value, nullptr, nullptr);
    else
        hipLaunchKernelGGL(k_heads_fc<6>, grid, block, 0, (hipStream_t)stream, work, n, params,
                           L, logits, value, nullptr, nullptr);
    return hipGetLastError() == hipSuccess ? RVZ_OK : RVZ_EHIP;
}

// trunk_split, then the FC heads on the f32 matrix cores (the product's k_heads_mfma)
int rvz_resnet_fwd_split(int32_t board, const float* x, int32_t n, const float* params,
                         const uint16_t* wsplit, int32_t filters, int32_t blocks, float* work,
                         float* logits, float* value, void* stream) {
    if (!logits || !value) return RVZ_EINVAL;
    const int rc =
        rvz_resnet_trunk_split(board, x, n, params, wsplit, filters, blocks, work, stream);
    if (rc != RVZ_OK || n == 0) return rc;
    const Layout L = make_layout(filters, blocks, board);
    const dim3 grid((n + 15) / 16), block(256);
    if (board == 8)
        hipLaunchKernelGGL(k_heads_mfma<8>, grid, block, 0, (hipStream_t)stream, work, n, params,
                           L, logits, value, nullptr, nullptr);
    else
        hipLaunchKernelGGL(k_heads_mfma<6>, grid, block, 0, (hipStream_t)stream, work, n, params,
                           L, logits, value, nullptr, nullptr);
    return hipGetLastError() == hipSuccess ? RVZ_OK : RVZ_EHIP;
}

}  // extern "C"
