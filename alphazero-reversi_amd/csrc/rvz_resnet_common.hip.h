// rvz_resnet_common.hip.h — pieces of the policy/value ResNet kernels shared by the product
// evaluator (csrc/rvz_resnet.hip, k_resnet_h2 + k_heads_mfma) and the A/B / cross-check build
// (tools/alt/rvz_resnet_alt.hip): the packed parameter layout, the 1x1 head convs, the batched FC
// heads on the f32 matrix cores, the compacted-batch row test and the phase-timing stamps.
// Packed parameter buffer (fp32, BN folded by rvz.network.pack_resnet_params; every segment starts
// 16-byte aligned; offsets in make_layout):
//   stem_w[F][27] (k = tap*3 + ch), stem_b[F], res_w[2NB][9][F(n)][F(k)], res_b[2NB][F],
//   pol_w[2][F], pol_b[2], pfc_w[65][128] (in = c*64 + px), pfc_b[65], val_w[F], val_b[1],
//   vfc1_w[256][64], vfc1_b[256], vfc2_w[256], vfc2_b[1].
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/rvz.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

struct Layout {
    int64_t stem_w, stem_b, res_w, res_b, pol_w, pol_b, pfc_w, pfc_b, val_w, val_b, vfc1_w,
        vfc1_b, vfc2_w, vfc2_b, total;
};

__host__ __device__ inline int64_t al4(int64_t o) { return (o + 3) & ~int64_t(3); }

__host__ __device__ inline Layout make_layout(int F, int NB, int BS = 8) {
    Layout L;
    const int cells = BS * BS;
    int64_t o = 0;
    L.stem_w = o; o = al4(o + (int64_t)F * 27);
    L.stem_b = o; o = al4(o + F);
    L.res_w = o;  o = al4(o + (int64_t)2 * NB * 9 * F * F);
    L.res_b = o;  o = al4(o + (int64_t)2 * NB * F);
    L.pol_w = o;  o = al4(o + 2 * F);
    L.pol_b = o;  o = al4(o + 2);
    L.pfc_w = o;  o = al4(o + (int64_t)(cells + 1) * 2 * cells);
    L.pfc_b = o;  o = al4(o + cells + 1);
    L.val_w = o;  o = al4(o + F);
    L.val_b = o;  o = al4(o + 1);
    L.vfc1_w = o; o = al4(o + 256 * cells);
    L.vfc1_b = o; o = al4(o + 256);
    L.vfc2_w = o; o = al4(o + 256);
    L.vfc2_b = o; o = al4(o + 1);
    L.total = o;
    return L;
}

// heads (network.py:104-117), part 1: the 1x1 convs (BN folded) + ReLU of both heads, in one
// pass over the activations: lane = pixel, wave = (board, channel group), partial sums per group
// through LDS (`part`, the free ping-pong buffer) added in a fixed order. Writes, per board b
// (cells = BS*BS), hpv(b)[0 .. 2 cells) = the policy planes (NCHW flatten, the FC's input order)
// and hpv(b)[2 cells .. 3 cells) = the value plane. A BS < 8 board sits in the top-left corner
// of the 8x8 pixel grid.
// The barrier the evaluator device functions use between their phases: the workgroup's
// (__syncthreads) by default; the fused kernel's teams pass their own (a 4-wave barrier in LDS)
struct BarWG {
    __device__ __forceinline__ void operator()() const { __syncthreads(); }
};
template <int F, int NBOARD, int NTHR, int BS = 8, bool PACKED = false, bool ILV = false, class Act,
          class Out, class Bar = BarWG>
__device__ __forceinline__ void head_convs(const Act& act, float* part,
                                           const float* __restrict__ prm, const Layout& L,
                                           const Out& hpv, int tid, const Bar& bar = Bar{}) {
    constexpr int NW = NTHR / 64, CG = NW / NBOARD, CPG = F / CG;
    static_assert(CPG % 8 == 0, "8-channel reads");
    const int lane = tid & 63;
    {
        const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
        // PACKED: board b's cells are act rows b * BS^2 + cell (h2); else the 8x8 grid
        const int b = wave % NBOARD, cg = wave / NBOARD, row = b * 64 + lane;
        // ILV (k_resnet_h2, two 8x8 boards): cell (r, c) of board b is act row r * 16 + b * 8 + c
        const int arow = ILV ? (lane >> 3) * 16 + b * 8 + (lane & 7)
                             : (PACKED ? b * BS * BS + lane : row);
        const bool on = !PACKED || lane < BS * BS;
        const float* w0 = prm + L.pol_w + cg * CPG;
        const float* w1 = w0 + F;
        const float* w2 = prm + L.val_w + cg * CPG;
        float p0 = 0.0f, p1 = 0.0f, p2 = 0.0f;
#pragma unroll
        for (int k8 = 0; k8 < CPG / 8; ++k8) {
            if (!on) break;
            float v[8];
            act.load8(arow, cg * CPG + 8 * k8, v);
            const float mb = act.mul(b);              // the board's activation scale (1: none)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                v[j] *= mb;
                p0 = fmaf(v[j], w0[8 * k8 + j], p0);
                p1 = fmaf(v[j], w1[8 * k8 + j], p1);
                p2 = fmaf(v[j], w2[8 * k8 + j], p2);
            }
        }
        part[(cg * 3 + 0) * NBOARD * 64 + row] = p0;
        part[(cg * 3 + 1) * NBOARD * 64 + row] = p1;
        part[(cg * 3 + 2) * NBOARD * 64 + row] = p2;
    }
    bar();
    constexpr int CELLS = BS * BS;
    for (int o = tid; o < NBOARD * 3 * CELLS; o += NTHR) {
        const int c2 = o / (NBOARD * CELLS), rem = o % (NBOARD * CELLS);
        const int b = rem / CELLS, cell = rem % CELLS;
        const int row = b * 64 + (PACKED ? cell : (cell / BS) * 8 + cell % BS);
        float acc = 0.0f;
#pragma unroll
        for (int g = 0; g < CG; ++g) acc += part[(g * 3 + c2) * NBOARD * 64 + row];
        const float bias = c2 < 2 ? prm[L.pol_b + c2] : prm[L.val_b];
        hpv.store(b, c2 * CELLS + cell, fmaxf(acc + bias, 0.0f));
    }
}
struct HeadsLds {        // hpv rows in LDS
    float* p;
    __device__ void store(int b, int i, float v) const { p[b * 192 + i] = v; }
};
struct HeadsGlobal {     // hpv rows in the global workspace of rvz_resnet_fwd_split
    float* p;
    int g0, n_boards;
    __device__ void store(int b, int i, float v) const {
        if (g0 + b < n_boards) p[(size_t)(g0 + b) * 192 + i] = v;
    }
};

// RVZ_PLAY_TIMING (tools/exp_play_phases.py): shader clocks of a fused trunk pass's parts per
// workgroup, [0] zero rows + stem (to its barrier), [1] [0] + the residual tower, [2] 1x1 head
// convs, [3] passes; of the FC heads (held weights), [4] to the weights' arrival, [5] the rest
#ifdef RVZ_PLAY_TIMING
__device__ unsigned long long g_pass_t[16384][6];
#define PASS_NOW(t) const unsigned long long t = __builtin_amdgcn_s_memtime()
#define PASS_ADD(i, v) if (threadIdx.x == 0 && blockIdx.x < 16384) g_pass_t[blockIdx.x][i] += (v)
#else
#define PASS_NOW(t)
#define PASS_ADD(i, v)
#endif

// a compacted leaf batch (include/rvz.h RVZ_LIVE_STRIPE): is the row past its stripe's live count?
__device__ __forceinline__ bool row_dead(const int32_t* __restrict__ n_live, int row) {
    return n_live && row % RVZ_LIVE_STRIPE >= n_live[row / RVZ_LIVE_STRIPE * RVZ_LIVE_PITCH];
}

// heads, part 2 on the f32 matrix cores (v_mfma_f32_16x16x4_f32: exact fp32 products, fp32
// accumulation — the arithmetic of an fp32 GEMM), 16 boards per workgroup: D = W X^T with rows =
// output units (16-unit tiles: value fc1 16 tiles, policy fc ceil((cells+1)/16)), columns = the
// 16 boards. The K order is permuted (step 4j + i uses k = 16j + 4g + i for lane group
// g = lane >> 4), so a lane loads 4 consecutive k of its weight row (f32x4, L2) and of its
// board's input row (ds_read_b128) per 4 MFMAs. Value fc2 (256 -> 1) + tanh reduce the fc1 tiles
// through registers, lane shuffles and 64 floats of LDS.
// RVZ_HEADS_STREAM 1 (default): the weight fragments are streamed through buffer loads,
// RVZ_HEADS_PD steps (one f32x4 and 4 MFMAs each) ahead, instead of all held at once (148 VGPRs).
// The kernel then fits in 76 VGPRs, so its waves run beside two trunk waves (2 x 216) instead of
// waiting for a trunk workgroup to end: C2 +0.3% (3 alternating whole-bench pairs, 727.0k ->
// 729.5k, profiles/r02z_ab_heads.txt; PD 6+ spills under the 80-VGPR cap).
#ifndef RVZ_HEADS_STREAM
#define RVZ_HEADS_STREAM 1
#endif
#ifndef RVZ_HEADS_PD
#define RVZ_HEADS_PD 4
#endif
#ifndef RVZ_HEADS_WPE
#define RVZ_HEADS_WPE 6      // waves per SIMD the heads are built for (6: <= 80 VGPRs)
#endif
#if RVZ_HEADS_STREAM
#define RVZ_HEADS_ATTR __attribute__((amdgpu_waves_per_eu(RVZ_HEADS_WPE)))
#else
#define RVZ_HEADS_ATTR
#endif
// Rows of the 16 board columns of one FC-heads pass: column b is row s0 + b (< n) of the
// workspace / outputs (k_heads_mfma), or row rows[b] (>= 0; an LDS list: k_play)
struct HeadRowsRange {
    int s0, n;
    __device__ int row(int b) const { return s0 + b < n ? s0 + b : -1; }
};
struct HeadRowsList {
    const int* rows;   // [16], -1: no board
    __device__ int row(int b) const { return rows[b]; }
};
__host__ __device__ constexpr int heads_in_floats(int BS) {
    return 16 * ((2 * BS * BS + 15) / 16 * 16 + (BS * BS + 15) / 16 * 16 + 4);
}
// One pass of the FC heads over 16 board columns (the body of k_heads_mfma): `in` is
// heads_in_floats(BS) floats of LDS, vpart 64; both free on entry. Ends with a barrier.
// STREAM: the weight fragments streamed RVZ_HEADS_PD steps ahead (76 VGPRs: k_heads_mfma's
// waves fit beside two trunk waves), or all issued up front (one L2 round trip; ~148 VGPRs: the
// fused k_play, whose register budget is the trunk's)
// COPY: the 16 rows are copied from the workspace into `in`; false: they are there already
// (the fused kernel's head convs wrote them, HeadsInLds)
// INROWS < 16: `in` holds INROWS rows and column c reads row c % INROWS (columns past the
// rows are not stored: their outputs are discarded)
template <int BS, class Rows, bool STREAM = RVZ_HEADS_STREAM != 0, bool COPY = true,
          int INROWS = 16, class Bar = BarWG>
__device__ __forceinline__ void heads_fc16(const float* __restrict__ work, const Rows& rmap,
                                           const float* __restrict__ prm, const Layout& L,
                                           float* __restrict__ logits, float* __restrict__ value,
                                           float* __restrict__ in, float (*vpart)[16],
                                           int tid = threadIdx.x, const Bar& bar = Bar{}) {
    constexpr int CELLS = BS * BS, PIN = 2 * CELLS, POUT = CELLS + 1;
    constexpr int VK = (CELLS + 15) / 16 * 16, PK = (PIN + 15) / 16 * 16;
    constexpr int PT = (POUT + 15) / 16, ROW = PK + VK + 4;   // +4: 16-B aligned, spread banks
    constexpr int VJ = VK / 16, PJ = PK / 16, VTW = 256 / 16 / 4, PTW = (PT + 3) / 4;
    static_assert(CELLS % 4 == 0 && PIN % 4 == 0, "f32x4 rows");
    static_assert(16 * ROW == heads_in_floats(BS), "LDS size");
    const int lane = tid & 63, wave = tid >> 6;
    const int col = lane & 15, grp = lane >> 4;
    const int grow = rmap.row(col);                  // this lane's board column: its row
    PASS_NOW(th0);

    // the wave's weight steps in order: value fc1 tiles wave + 4m (VJ steps each), then policy
    // tiles wave + 4m (PJ steps each); step s = one f32x4 of the A row (unit 16 t + col,
    // k = 16 j + 4 grp .. +3)
    constexpr int NSV = VTW * VJ, NS = NSV + PTW * PJ, D = RVZ_HEADS_PD < NS ? RVZ_HEADS_PD : NS;
    // buffer loads: the lane's part of the address is one VGPR, the step's part (wave-uniform) the
    // scalar soffset, so no 64-bit address per step is kept live
    const __amdgpu_buffer_rsrc_t rw =
        __builtin_amdgcn_make_buffer_rsrc((void*)prm, (short)0, (int)(L.total * 4), 0x00020000);
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    auto load_step = [&](int s) -> f32x4 {
        if (s < NSV) {
            const int m = s / VJ, j = s % VJ;
            const int so = (int)(L.vfc1_w + (16 * (wv + 4 * m)) * CELLS + 16 * j) * 4;
            return 16 * j + 4 * grp < CELLS
                       ? __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                       rw, (col * CELLS + 4 * grp) * 4, so, 0))
                       : f32x4{};
        }
        const int m = (s - NSV) / PJ, j = (s - NSV) % PJ, o = 16 * (wv + 4 * m) + col;
        const int so = (int)(L.pfc_w + (16 * (wv + 4 * m)) * PIN + 16 * j) * 4;
        return (o < POUT && 16 * j + 4 * grp < PIN)
                   ? __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                   rw, (col * PIN + 4 * grp) * 4, so, 0))
                   : f32x4{};
    };
    f32x4 wq[D];
    if constexpr (STREAM) {
#pragma unroll
        for (int s = 0; s < D; ++s) wq[s] = load_step(s);
    }

    // every weight fragment of this wave's tiles, issued before anything waits: value fc1 tiles
    // wave + 4m, policy tiles wave + 4m (A row = unit 16 t + col, k = 16 j + 4 grp .. +3)
    f32x4 av[VTW][VJ], ap[PTW][PJ];
    if constexpr (!STREAM) {
#pragma unroll
    for (int m = 0; m < VTW; ++m) {
        const float* wr = prm + L.vfc1_w + (size_t)(16 * (wave + 4 * m) + col) * CELLS + 4 * grp;
#pragma unroll
        for (int j = 0; j < VJ; ++j)
            av[m][j] = 16 * j + 4 * grp < CELLS ? *reinterpret_cast<const f32x4*>(wr + 16 * j)
                                                : f32x4{};
    }
#pragma unroll
    for (int m = 0; m < PTW; ++m) {
        const int o = 16 * (wave + 4 * m) + col;
        const float* wr = prm + L.pfc_w + (size_t)o * PIN + 4 * grp;
#pragma unroll
        for (int j = 0; j < PJ; ++j)
            ap[m][j] = (o < POUT && 16 * j + 4 * grp < PIN)
                           ? *reinterpret_cast<const f32x4*>(wr + 16 * j) : f32x4{};
    }
    }

    if constexpr (COPY) {   // the 16 workspace rows into LDS, 16 B per load, all in flight
        // (policy planes at k < PIN, the value plane at PK.., zeros between)
        constexpr int RQ = (PK + VK) / 4, NQ = 16 * RQ / 256;
        static_assert(16 * RQ % 256 == 0 && PK % 4 == 0 && ROW % 4 == 0, "whole float4 rounds");
        f32x4 v[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int i = tid + 256 * q, b = i / RQ, k = 4 * (i % RQ);
            const int src = k < PIN ? k : (k >= PK && k - PK < CELLS ? PIN + k - PK : -1);
            const int rb = rmap.row(b);
            v[q] = rb >= 0 && src >= 0
                       ? *reinterpret_cast<const f32x4*>(work + (size_t)rb * 192 + src)
                       : f32x4{};
        }
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int i = tid + 256 * q, b = i / RQ, k = 4 * (i % RQ);
            *reinterpret_cast<f32x4*>(in + b * ROW + k) = v[q];
        }
    }
    bar();
#ifdef RVZ_PLAY_TIMING
    if constexpr (!STREAM) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    PASS_NOW(th1);
    if constexpr (!STREAM) PASS_ADD(4, th1 - th0);
    const float* inb = in + (col % INROWS) * ROW + 4 * grp;
    float vp = 0.0f;
    if constexpr (STREAM) {
    f32x4 acc = {};
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        __builtin_amdgcn_sched_barrier(0);   // keep each step's load in its step (no hoisting)
        const f32x4 w = wq[s % D];
        if (s + D < NS) wq[s % D] = load_step(s + D);
        const bool val = s < NSV;
        const int m = val ? s / VJ : (s - NSV) / PJ, j = val ? s % VJ : (s - NSV) % PJ;
        const int t = wave + 4 * m;
        if (j == 0) acc = f32x4{};
        if (val || t < PT) {
            const f32x4 bx = *reinterpret_cast<const f32x4*>(inb + (val ? PK : 0) + 16 * j);
#pragma unroll
            for (int i = 0; i < 4; ++i)
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(w[i], bx[i], acc, 0, 0, 0);
        }
        if (val && j == VJ - 1) {
            // bias and fc2 weights of the tile's 4 rows: one 16-B buffer load each
            const int ub = 16 * (wv + 4 * m);
            const f32x4 b1 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                 rw, 16 * grp, (int)(L.vfc1_b + ub) * 4, 0));
            const f32x4 w2 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                 rw, 16 * grp, (int)(L.vfc2_w + ub) * 4, 0));
#pragma unroll
            for (int r = 0; r < 4; ++r) vp = fmaf(fmaxf(acc[r] + b1[r], 0.0f), w2[r], vp);
            if (m == VTW - 1) {
                vp += __shfl_xor(vp, 16);
                vp += __shfl_xor(vp, 32);
                if (grp == 0) vpart[wave][col] = vp;
            }
        }
        if (!val && j == PJ - 1 && t < PT) {
            const f32x4 pb = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                 rw, 16 * grp, (int)(L.pfc_b + 16 * t) * 4, 0));
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int oo = 16 * t + 4 * grp + r;
                if (oo < POUT && grow >= 0) logits[(size_t)grow * POUT + oo] = acc[r] + pb[r];
            }
        }
    }
    } else {
    // value fc1 tile epilogue (+ bias, ReLU) into the fc2 partial
    auto value_tile = [&](int m, const f32x4& acc) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {                // D row = unit 16t + 4grp + r, col = board
            const int uu = 16 * (wave + 4 * m) + 4 * grp + r;
            vp = fmaf(fmaxf(acc[r] + prm[L.vfc1_b + uu], 0.0f), prm[L.vfc2_w + uu], vp);
        }
    };
    auto policy_tile = [&](int t, const f32x4& acc) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int oo = 16 * t + 4 * grp + r;
            if (oo < POUT && grow >= 0) logits[(size_t)grow * POUT + oo] = acc[r] + prm[L.pfc_b + oo];
        }
    };
    // value fc1 (+ bias, ReLU) and its fc2 partial
#pragma unroll
    for (int m = 0; m < VTW; ++m) {
        f32x4 acc = {};
#pragma unroll
        for (int j = 0; j < VJ; ++j) {
            const f32x4 bx = *reinterpret_cast<const f32x4*>(inb + PK + 16 * j);
#pragma unroll
            for (int i = 0; i < 4; ++i)
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[m][j][i], bx[i], acc, 0, 0, 0);
        }
        value_tile(m, acc);
    }
    vp += __shfl_xor(vp, 16);
    vp += __shfl_xor(vp, 32);
    if (grp == 0) vpart[wave][col] = vp;
    // policy fc
#pragma unroll
    for (int m = 0; m < PTW; ++m) {
        const int t = wave + 4 * m;
        if (t >= PT) break;
        f32x4 acc = {};
#pragma unroll
        for (int j = 0; j < PJ; ++j) {
            const f32x4 bx = *reinterpret_cast<const f32x4*>(inb + 16 * j);
#pragma unroll
            for (int i = 0; i < 4; ++i)
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ap[m][j][i], bx[i], acc, 0, 0, 0);
        }
        policy_tile(t, acc);
    }
    }
    bar();
    if (tid < 16) {
        const int rt = rmap.row(tid);
        if (rt >= 0)
            value[rt] = tanhf(((vpart[0][tid] + vpart[1][tid]) + (vpart[2][tid] + vpart[3][tid])) +
                              prm[L.vfc2_b]);
    }
    bar();
    PASS_NOW(th2);
    if constexpr (!STREAM) PASS_ADD(5, th2 - th1);
}

template <int BS>
__global__ __launch_bounds__(256) RVZ_HEADS_ATTR void k_heads_mfma(
    const float* __restrict__ work, int n, const float* __restrict__ prm, Layout L,
    float* __restrict__ logits, float* __restrict__ value, const int32_t* __restrict__ n_live,
    uint32_t* __restrict__ stamp_ctr) {
    // bench.py: the trunk launch before this one is complete; advance its stamp ring
    if (stamp_ctr && blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(stamp_ctr, 1u);
    if (row_dead(n_live, (int)blockIdx.x * 16)) return;    // the workgroup's rows are all dead
    __shared__ __attribute__((aligned(16))) float in[heads_in_floats(BS)];
    __shared__ float vpart[4][16];
    heads_fc16<BS>(work, HeadRowsRange{(int)blockIdx.x * 16, n}, prm, L, logits, value, in, vpart);
}


#ifdef RVZ_PHASE_TIMING   // tools/phase_timing.py: per-workgroup s_memtime at phase boundaries
__device__ uint64_t g_phase[65536][8];
__device__ uint64_t g_rt[65536][2];   // s_memrealtime (100 MHz) at start / end
__device__ uint64_t g_wave[65536][16];
#define PHASE(i) \
    if (threadIdx.x == 0 && blockIdx.x < 65536) g_phase[blockIdx.x][i] = __builtin_amdgcn_s_memtime()
#define RT(i) \
    if (threadIdx.x == 0 && blockIdx.x < 65536) g_rt[blockIdx.x][i] = __builtin_amdgcn_s_memrealtime()
__device__ uint64_t g_stem[65536][8];
__device__ uint32_t g_hwid[65536][2];   // HW_ID (CU, SE, ...), XCC_ID of each workgroup
#define HWID() \
    if (threadIdx.x == 0 && blockIdx.x < 65536) { \
        g_hwid[blockIdx.x][0] = __builtin_amdgcn_s_getreg((31 << 11) | 4); \
        g_hwid[blockIdx.x][1] = __builtin_amdgcn_s_getreg((31 << 11) | 20); \
    }
#define STEM_T(i) \
    if (threadIdx.x == 0 && blockIdx.x < 65536) g_stem[blockIdx.x][i] = __builtin_amdgcn_s_memtime()
#define WAVE_T(i) \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 65536) \
        g_wave[blockIdx.x][(threadIdx.x >> 6) + 8 * (i)] = __builtin_amdgcn_s_memtime()
#else
#define PHASE(i)
#define HWID()
#define STEM_T(i)
#define WAVE_T(i)
#define RT(i)
#endif

// sched_group_barrier pattern: NM MFMAs, the first ND gaps get one LDS read, the next NV one
// global load
template <int I, int NM, int ND, int NV>
__device__ __forceinline__ void interleave_loads() {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    if constexpr (I < ND) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    else if constexpr (I < ND + NV) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    if constexpr (I + 1 < NM) interleave_loads<I + 1, NM, ND, NV>();
}

}  // namespace
