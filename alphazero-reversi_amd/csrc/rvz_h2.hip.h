// rvz_h2.hip.h — the h2 leaf-evaluator trunk (fp32 as a two-part f16 split on the f16 matrix
// cores) as device functions: one pass of a workgroup over NBOARD boards (h2_pass) — stem,
// residual tower and the 1x1 head convs, activations resident in LDS. Used by the trunk kernel
// (csrc/rvz_resnet.hip, k_resnet_h2: one pass per workgroup over a leaf batch) and by the fused
// self-play kernel (csrc/rvz_engine.hip, k_play: a workgroup's own games' leaves, pass after pass).
#pragma once
#include "rvz_resnet_common.hip.h"

namespace {

// =============================================================================================
// h2 kernel: fp32 as an exact two-part f16 split, three partial products (rvz_resnet_fwd_h2)
//
// Numerics. f16 carries 11 significant bits; x = x0 + x1 + r with x0 = f16(x), x1 = f16(x - x0)
// (x - x0 is exact in fp32) and |r| <= 2^-22 |x|. Each conv product is accumulated as
// x0w0 + x0w1 + x1w0 in ONE fp32 accumulator (v_mfma_f32_16x16x32_f16, the bf16 rate); the
// dropped x1w1 and the residuals are <= ~2^-21 |x w|. Summed over K = 9F products with fp32
// accumulation, the error is that of an fp32 GEMM (tools/emu_split.py: 0.8-1.5x plain fp32's
// error against fp64 on 6x64 / 10x128 nets; tests/test_gpu_network.py measures the kernel).
// Range: f16 is normal in [2^-14, 65504]. Weights are scaled per output channel by a power of two
// so that the channel's max |w| lands in [2^14, 2^15) (the epilogue multiplies the accumulator by
// the exact inverse), so every weight >= 2^-17 of its channel's max keeps 22 bits. Activations are
// not scaled: |x| >= 2^-3 keeps 22 bits, smaller ones an absolute error <= 2^-25 (f16 subnormal
// step of x1); |x| >= 65520 overflows to inf (a trained net's activations are far below; the
// kernel stores 1 in work[n * 192] (the overflow word, a float) if any activation overflowed).
// Half the MFMAs of the 3-part bf16 scheme (3 products instead of 6) and 2/3 of its LDS: 66 KB
// per workgroup, so two workgroups share a CU and overlap one's epilogue/barrier with the
// other's k-loop.
//
// LDS: act[2 buffers][2 parts][F/32 k-step planes][NBOARD*64 + 8 rows][32 halves]; rows
// NBOARD*64 .. +7 are zero. A row of a plane is 4 16-byte slots; slot q of row r is stored at
// slot q ^ ((r >> 1) & 3). An off-board tap of target row r reads zero row NBOARD*64 + (r & 7),
// which has r's bank placement. Bank analysis (ds_read_b128 lane groups {0-3,12-15,20-27},
// {4-11,16-19,28-31} +32; ds_write_b64 groups of 16 contiguous lanes; MI355X_MICROARCH.md §LDS),
// checked exhaustively over every tap, tile and both board sizes by tools/lds_banks.py: the B
// operand reads are conflict-free (4 LDS cycles per read), the epilogue's 8-byte writes 2-way,
// the minimum for 16 pixels x one channel quad in 64-byte rows.
// The k-step and the part are immediate offsets of one address per (pixel tile, tap).
// Wave tiles as k_resnet_split on 16x16x32: CTW = 2 channel tiles x PTW = 4 pixel tiles.
// Weight blob (rvz_resnet_h2_weights), uint16 units:
//   [trunk frags: layer][tap][kstep][part][ctile][lane][8]  (pre-scaled f16 parts)
//   [H2_PAD k-steps of zeros: the prefetch past the last layer]
//   [stem frags: part][ctile][lane][8]  (K = 27 padded to 32, k = tap*3 + ch)
//   [inverse scales: float[1 + 2*NB][F]: stem, then the trunk layers]

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2v __attribute__((ext_vector_type(2)));

#ifndef RVZ_H2_PD
#define RVZ_H2_PD 2          // weight prefetch distance, k-steps
#endif
#ifndef RVZ_H2_APD
#define RVZ_H2_APD 1         // activation prefetch distance, k-steps
#endif
#ifndef RVZ_H2_OCC
#define RVZ_H2_OCC 2         // workgroups per CU the register budget is sized for
#endif
#ifndef RVZ_H2_ILV
#define RVZ_H2_ILV 1         // 8x8, 2 boards per workgroup: row-interleaved pixels, edge taps skipped
#endif                       // (0: board-major pixels, every tap computed)

constexpr int H2_K = 32, H2_TM = 16, H2_TN = 16;

__host__ __device__ inline int64_t h2_layer_elems(int F) { return (int64_t)9 * F * F * 2; }
__host__ __device__ inline int64_t h2_kstep_elems(int F) { return (int64_t)2 * F * H2_K; }
// zero k-steps after the last layer: the weight prefetch of the next (absent) layer reads them.
// (A mirrored wave (ILV) starts a layer at tap 8; its prefetch past the last layer lands in the
// stem / scale words or past the blob, where the buffer descriptor's range check returns 0: the
// values are discarded either way.)
__host__ __device__ inline int64_t h2_pad_ksteps(int) { return 4; }
static_assert(RVZ_H2_PD <= 4, "prefetch stays inside the padded blob");
__host__ __device__ inline int64_t h2_stem_off(int F, int NB) {
    return 2 * NB * h2_layer_elems(F) + h2_pad_ksteps(F) * h2_kstep_elems(F);
}
__host__ __device__ inline int64_t h2_scale_off(int F, int NB) {   // uint16 units, 16-B aligned
    return h2_stem_off(F, NB) + (int64_t)2 * F * H2_K;
}
__host__ __device__ inline int64_t h2_blob_elems(int F, int NB) {
    return h2_scale_off(F, NB) + (int64_t)2 * (1 + 2 * NB) * F;
}

// x == h0 + h1 + r, |r| <= 2^-22 |x| for |x| in the f16 normal range (round to nearest even)
__device__ __forceinline__ void split2x2(f32x2 x, uint32_t& h0, uint32_t& h1) {
    const f16x2v a = __builtin_convertvector(x, f16x2v);
    const f32x2 r = x - __builtin_convertvector(a, f32x2);
    const f16x2v b = __builtin_convertvector(r, f16x2v);
    h0 = __builtin_bit_cast(uint32_t, a);
    h1 = __builtin_bit_cast(uint32_t, b);
}
__device__ __forceinline__ float h16f(uint16_t h) {
    return (float)__builtin_bit_cast(_Float16, h);
}

// Board geometry of a workgroup: NB boards of BS x BS cells packed row-major, pixel row
// px = b * BS^2 + r * BS + c (8x8: b * 64 + r * 8 + c; a 6x6 board takes 36 rows, not the 64 of
// an embedding in the 8x8 grid), rounded up to whole 16-pixel MFMA tiles; rows past the boards
// are padding (no valid tap, never read), up to a multiple of RND (whole pixel tiles for every
// wave: 16 x the waves along the pixels).
// ILV (two 8x8 boards): row-interleaved, px = r * 16 + b * 8 + c, so a 16-pixel tile is board
// row r of both boards and the taps of row 0 (dr = -1) and row 7 (dr = +1) leave the boards for
// the whole tile: those tile x tap products are skipped, 1/12 of the conv MFMAs (conv_h2).
template <int NB, int BS, int RND, bool ILV = false>
struct GeoH {
    static constexpr int PPB = BS * BS;
    static constexpr int NVALID = NB * PPB;
    static constexpr int NPIX = (NVALID + RND - 1) / RND * RND;
    static constexpr int RS = ILV ? NB * BS : BS;    // pixel-row stride of a board row
    static_assert(!ILV || (NB == 2 && BS == 8), "interleaved rows: two 8x8 boards");
    static __device__ __forceinline__ int cell_of(int px) {
        return ILV ? (px >> 4) * 8 + (px & 7) : px % PPB;
    }
    static __device__ __forceinline__ int board_of(int px) { return ILV ? (px >> 3) & 1 : px / PPB; }
    static __device__ __forceinline__ int row_of(int b, int cell) {
        return ILV ? (cell >> 3) * 16 + b * 8 + (cell & 7) : b * PPB + cell;
    }
    // the 3x3 taps of pixel px that stay on its board (bit t = tap (t/3 - 1, t%3 - 1))
    static __device__ __forceinline__ unsigned taps(int px) {
        const int cell = cell_of(px), r = cell / BS, c = cell % BS;
        unsigned m = 0;
#pragma unroll
        for (int t = 0; t < 9; ++t)
            if ((unsigned)(r + t / 3 - 1) < (unsigned)BS && (unsigned)(c + t % 3 - 1) < (unsigned)BS)
                m |= 1u << t;
        return px < NVALID ? m : 0u;
    }
    static __device__ __forceinline__ int tap_offset(int t) { return (t / 3 - 1) * RS + (t % 3 - 1); }
};

template <int F, int NPIX>
struct CfgH {
    static constexpr int ZROW = NPIX;                // first of the 8 zero rows
    static constexpr int KS = F / H2_K;              // k-step planes of 32 channels
    static constexpr int KSP = (ZROW + 8) * H2_K;    // halves per k-step plane
    static constexpr int PLANE = KS * KSP;           // halves per part
    static constexpr int ACT = 2 * PLANE;            // halves per buffer
    static constexpr int BYTES = 2 * ACT * 2;
    static constexpr int NIT = 9 * KS;
    static constexpr int CT = F / H2_TM;
    static_assert((PLANE * 2) % 16 == 0 && (KSP * 2) % 16 == 0, "16-byte aligned planes");
    static_assert(BYTES <= 160 * 1024, "fits the LDS of a CU");
    // halves offset of (row, k-step plane ks, 8-channel slot q in 0..3)
    static __device__ __forceinline__ int at(int row, int ks, int q) {
        return ks * KSP + row * H2_K + 8 * (q ^ ((row >> 1) & 3));
    }
};

// activation reader for the heads (join of the two parts)
template <int F, int NPIX>
struct ActH2 {
    const uint16_t* p;
    __device__ void load8(int row, int k0, float (&v)[8]) const {
        typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));
        const int o = CfgH<F, NPIX>::at(row, k0 / H2_K, (k0 % H2_K) >> 3);
        const u16x8 a = *reinterpret_cast<const u16x8*>(p + o);
        const u16x8 b = *reinterpret_cast<const u16x8*>(p + CfgH<F, NPIX>::PLANE + o);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = h16f(a[j]) + h16f(b[j]);
    }
};

// A wave's output tiles: CTW channel tiles from ct0 and PTW pixel tiles. ilv (GeoH ILV): pixel
// group 0 holds board rows 0-3 (tile u = row u), group 1 rows 7-4 (tile u = row 7 - u), so tile 0
// is the edge row of either group.
template <int F, int CTW, int PTW>
struct WaveTilesH {
    static constexpr int CG = F / (CTW * H2_TM);
    int ct0, px[PTW];
    __device__ WaveTilesH(int wave, int lane, bool ilv = false) {
        ct0 = (wave % CG) * CTW;
        const int pg = wave / CG, pt0 = pg * PTW;
#pragma unroll
        for (int u = 0; u < PTW; ++u)
            px[u] = (ilv ? (pg ? 7 - u : u) : pt0 + u) * H2_TN + lane % H2_TN;
    }
};

// Weight fragments are read through a buffer descriptor over the whole blob: the wave-uniform
// part of the address (layer, tap, k-step, part, channel tile) is the scalar soffset and the
// lane's 16-byte slot the only VGPR, so a mirrored wave's runtime tap order costs scalar adds.
// Reads past the blob return 0 (the descriptor's range check).
struct H2W {
    __amdgpu_buffer_rsrc_t r;
    __device__ H2W(const uint16_t* blob, int64_t elems)
        : r(__builtin_amdgcn_make_buffer_rsrc((void*)blob, (short)0, (int)(elems * 2), 0x00020000)) {}
    // f16x8 fragment at f16x8 index `idx` (wave-uniform) + this lane
    __device__ __forceinline__ f16x8 load(int idx, int lane) const {
        return __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16,
                                                                               idx * 16, 0));
    }
};
// f16x8 index of k-step `it` of a layer (it >= NIT: the next layer's) from the layer's base:
// [tap][kstep][part][ctile][lane]. mirror (ILV pixel group 1, RVZ_H2_MIRROR 1 or 2): the wave
// walks the tap rows in reverse, so both groups meet their edge taps at the same it.
#ifndef RVZ_H2_MIRROR
#define RVZ_H2_MIRROR 0      // 0: natural order, a skip window per pixel group (conv_h2);
#endif                       // 1: (dr, dc) -> (-dr, -dc); 2: rows only, (dr, dc) -> (-dr, dc)
// the natural tap a mirrored wave reads at iteration tap t
__host__ __device__ constexpr int h2_mirror_tap(int t) {
    return RVZ_H2_MIRROR == 1 ? 8 - t : (2 - t / 3) * 3 + t % 3;
}
template <int F>
__device__ __forceinline__ int h2_frag(int it, bool mirror) {
    constexpr int KS = F / H2_K, NIT = 9 * KS, CT = F / H2_TM, KSTEP = 2 * CT * 64;
    const int lay = it / NIT, itn = it % NIT, t = itn / KS, ks = itn % KS;
    const int tn = mirror ? h2_mirror_tap(t) : t;
    return (lay * NIT + tn * KS + ks) * KSTEP;
}

// RVZ_H2_SKIP_LDS 1: the skip input is re-read from LDS as its two parts (x0 + x1, 22 bits: the
// precision the conv inputs already carry; tools/emu_split.py f16x2_1acc_lds) at the place conv B
// overwrites it, instead of kept in 32 fp32 registers. With the mirrored tap order (216 vs 248
// VGPRs) that let a k_step or FC-heads wave (<= 80) share a SIMD with the two trunk waves:
// +0.9-1.6% per ply (profiles/r02s_ablib_skiplds.txt, r02u). Under the natural-order trunk
// (190 vs 220 VGPRs) the registers win: 0 (default) is +1.05% per ply
// (profiles/r02ap_ab_skipreg.txt); `k_act` (63) still fits beside two 220-VGPR waves, k_step and
// the heads capped at 72 measured the same (profiles/r02aq_ab_caps.txt).
#ifndef RVZ_H2_SKIP_LDS
#define RVZ_H2_SKIP_LDS 0
#endif
// RVZ_H2_W128 1: the epilogue stores 16 bytes per lane (ds_write_b128, one per tile) after a
// v_permlane16_swap exchange between lane quads, instead of two 8-byte stores (ds_write_b64),
// which are 2-way bank-conflicted in any slot swizzle: a 16-lane ds_write_b64 group is 16 pixels
// of one channel quad, which fill only 8 of the 16 8-byte bank positions modulo 32 banks. Eight
// contiguous lanes of a b128 store are 8 consecutive pixel rows of one part, whose slots
// (row mod 2, (row >> 1) & 3) cover the 32 banks once: conflict-free (tools/lds_banks.py).
// C2's geometry only (ILV: F = 64, two 8x8 boards; the callers pass W128 = RVZ_H2_W128 && ILV):
// at F = 128 and for three 6x6 boards the exchange's live registers push k_play from 256 / 255
// VGPRs into spills. Measured and NOT kept (r04n, profiles/r04n_*): k_play's LDS bank conflicts
// 10.7% -> 0.7% of LDS cycles, but C2 -0.8% on one box (3 alternating pairs, 1,042.4k vs
// 1,034.1k; 233 -> 239 VGPRs, +2.8% VALU): a 2-way ds_write_b64 costs 8 LDS-array cycles against
// its ~6 transfer cycles, while the swaps and the 13-cycle b128 transfer cost more.
#ifndef RVZ_H2_W128
#define RVZ_H2_W128 0
#endif
// RVZ_H2_PK 1: the epilogue's scale + bias fma and residual add on channel pairs (packed fp32
// VALU), per element the same operations in the same order. Measured and NOT kept (r04u,
// profiles/r04u_ab_pk.txt): the conv epilogue drops from ~144-194 to ~129-174 VALU instructions
// per wave, k_play 233 -> 235 VGPRs, C2 -0.3% on one box (3 alternating pairs): the epilogue's
// VALU already issues in the partner's MFMA shadow.
#ifndef RVZ_H2_PK
#define RVZ_H2_PK 0
#endif
// The trunk's register / prefetch knobs as a type (the fused kernels instantiate more than one):
// SKIP = RVZ_H2_SKIP_LDS, APD / PD = the activation / weight prefetch distances in k-steps
// LATE: the epilogue's bias and inverse scales are loaded after the k-loop instead of before it
// (16 fewer VGPRs held through the loop; the load's latency is then exposed at each epilogue)
template <bool SKIP_, int APD_, int PD_, bool LATE_ = false>
struct H2Knobs {
    static constexpr bool SKIP = SKIP_, LATE = LATE_;
    static constexpr int APD = APD_, PD = PD_;
    static_assert(PD_ >= 1 && PD_ <= 4 && APD_ >= 0, "prefetch distances");
};
#ifndef RVZ_H2_LATE_EPI
#define RVZ_H2_LATE_EPI 0
#endif
using H2Def = H2Knobs<RVZ_H2_SKIP_LDS != 0, RVZ_H2_APD, RVZ_H2_PD, RVZ_H2_LATE_EPI != 0>;
// the trunk at <= 168 VGPRs (three waves per SIMD): skip input from LDS, no activation prefetch,
// weights one k-step ahead (profiles/r04v_ab_trunk_register_diet.json: 166 VGPRs, 3.8% slower
// alone)
using H2Diet = H2Knobs<true, 0, 1>;
template <int CTW, int PTW>
struct EpiH {
    f32x4 bias[CTW], isc[CTW];       // per out-channel bias, inverse weight scale
    float res[CTW][PTW][4];          // the block input (fp32) of this lane's outputs (SKIP: unused)
};

template <int F, int CTW, int PTW>
__device__ __forceinline__ void load_epi(EpiH<CTW, PTW>& er, const float* __restrict__ bias,
                                         const float* __restrict__ isc,
                                         const WaveTilesH<F, CTW, PTW>& wt, int lane) {
#pragma unroll
    for (int c = 0; c < CTW; ++c) {
        const int n = (wt.ct0 + c) * H2_TM + 4 * (lane >> 4);
        er.bias[c] = *reinterpret_cast<const f32x4*>(bias + n);
        er.isc[c] = *reinterpret_cast<const f32x4*>(isc + n);
    }
}

// v = acc * isc + bias (+ skip), ReLU, split into the two parts: the lane holds 4 consecutive
// channels of one pixel per tile -> two 8-byte writes
template <int F, int NPIX, int CTW, int PTW, bool RES, bool KEEP, bool W128 = false,
          bool SKIP = RVZ_H2_SKIP_LDS != 0>
__device__ __forceinline__ void epilogue_h2(uint16_t* __restrict__ out,
                                            const f32x4 (&acc)[CTW][PTW], EpiH<CTW, PTW>& er,
                                            const WaveTilesH<F, CTW, PTW>& wt, int lane,
                                            bool& ovf) {
    using C = CfgH<F, NPIX>;
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int c = 0; c < CTW; ++c)
#pragma unroll
        for (int u = 0; u < PTW; ++u) {
            const int n0 = (wt.ct0 + c) * H2_TM + 4 * (lane >> 4);
            const int o = C::at(wt.px[u], n0 / H2_K, (n0 % H2_K) >> 3) + (n0 & 4);
            f16x4 s0, s1;
            if (RES && SKIP) {
                s0 = *reinterpret_cast<const f16x4*>(out + o);
                s1 = *reinterpret_cast<const f16x4*>(out + C::PLANE + o);
            }
            u32x2 d0, d1;
#pragma unroll
            for (int hf = 0; hf < 2; ++hf) {
                f32x2 v;
                if constexpr (RVZ_H2_PK && !SKIP) {
                    // the same per-element fma, add and max on channel pairs (v_pk_fma_f32,
                    // v_pk_add_f32: one instruction per two values)
                    const int j0 = 2 * hf;
                    v = __builtin_elementwise_fma(f32x2{acc[c][u][j0], acc[c][u][j0 + 1]},
                                                  f32x2{er.isc[c][j0], er.isc[c][j0 + 1]},
                                                  f32x2{er.bias[c][j0], er.bias[c][j0 + 1]});
                    if (RES) v = v + f32x2{er.res[c][u][j0], er.res[c][u][j0 + 1]};
                    v = f32x2{fmaxf(v[0], 0.0f), fmaxf(v[1], 0.0f)};
                    ovf |= v[0] >= 65520.0f;
                    ovf |= v[1] >= 65520.0f;
                    if constexpr (KEEP) {
                        er.res[c][u][j0] = v[0];
                        er.res[c][u][j0 + 1] = v[1];
                    }
                } else
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    const int j = 2 * hf + e;
                    float x = fmaf(acc[c][u][j], er.isc[c][j], er.bias[c][j]);
                    if (RES) {
                        if constexpr (SKIP) x += (float)s0[j] + (float)s1[j];
                        else x += er.res[c][u][j];
                    }
                    x = fmaxf(x, 0.0f);
                    ovf |= x >= 65520.0f;
                    if constexpr (KEEP && !SKIP) er.res[c][u][j] = x;
                    v[e] = x;
                }
                uint32_t h0, h1;
                split2x2(v, h0, h1);
                d0[hf] = h0;
                d1[hf] = h1;
            }
            if constexpr (W128) {
                // lane quads 2k and 2k+1 (rows 2k, 2k+1 of 16 lanes) hold channels n8..n8+3 and
                // n8+4..+7 of one pixel: v_permlane16_swap(d0, d1) moves the odd quad's part-0
                // half into the even quad's d1 and the even quad's part-1 half into the odd
                // quad's d0, so the even quad writes the 8 channels of part 0 and the odd quad
                // those of part 1, 16 bytes each
                typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const auto r = __builtin_amdgcn_permlane16_swap(d0[i], d1[i], false, false);
                    d0[i] = r[0];
                    d1[i] = r[1];
                }
                const int q = lane >> 4, n8 = (wt.ct0 + c) * H2_TM + 8 * (q >> 1);
                const int o8 = C::at(wt.px[u], n8 / H2_K, (n8 % H2_K) >> 3) + (q & 1) * C::PLANE;
                *reinterpret_cast<u32x4*>(out + o8) = u32x4{d0[0], d0[1], d1[0], d1[1]};
            } else {
                *reinterpret_cast<u32x2*>(out + o) = d0;
                *reinterpret_cast<u32x2*>(out + C::PLANE + o) = d1;
            }
        }
}

// RVZ_H2_HEADS_EPI 1: the last conv's epilogue computes the 1x1 head convs (policy 2, value 1
// output channels) from its fp32 outputs in registers instead of storing them to LDS for
// head_convs to read back: per lane, partial dot products over its 4 x CTW channels for each of
// its PTW pixels, reduced over the four lane groups (shuffles) and, through LDS, over the
// channel-group waves. Needs the skip input in registers (the output buffer holds the partials).
#ifndef RVZ_H2_HEADS_EPI
#define RVZ_H2_HEADS_EPI 0
#endif
struct HeadPart {          // the 1x1 head-conv weights (pol_w [2][F], val_w [F]) and LDS partials
    const float* pol;
    const float* val;
    float* part;           // [channel group][3][NPIX]
};
template <int F, int NPIX, int CTW, int PTW>
__device__ __forceinline__ void epilogue_heads(const f32x4 (&acc)[CTW][PTW], EpiH<CTW, PTW>& er,
                                               const WaveTilesH<F, CTW, PTW>& wt, int wave,
                                               int lane, const f32x4 (&hw)[3][CTW],
                                               float* __restrict__ part, bool& ovf) {
    constexpr int CG = WaveTilesH<F, CTW, PTW>::CG;
    float ph[PTW][3];
#pragma unroll
    for (int u = 0; u < PTW; ++u) {
        ph[u][0] = ph[u][1] = ph[u][2] = 0.0f;
#pragma unroll
        for (int c = 0; c < CTW; ++c)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                float x = fmaf(acc[c][u][j], er.isc[c][j], er.bias[c][j]) + er.res[c][u][j];
                x = fmaxf(x, 0.0f);
                ovf |= x >= 65520.0f;
#pragma unroll
                for (int o = 0; o < 3; ++o) ph[u][o] = fmaf(x, hw[o][c][j], ph[u][o]);
            }
    }
#pragma unroll
    for (int u = 0; u < PTW; ++u)
#pragma unroll
        for (int o = 0; o < 3; ++o) {
            float v = ph[u][o];
            v += __shfl_xor(v, 16);
            v += __shfl_xor(v, 32);
            if (lane < 16) part[((wave % CG) * 3 + o) * NPIX + wt.px[u]] = v;
        }
}

__device__ __forceinline__ f32x4 mfma_h(f16x8 a, f16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
// the three partial products, consecutive MFMAs on different accumulators
// (U0 = 1: pixel tile 0 skipped, its tap is off the boards for the whole tile)
// (issue order measured neutral: pixel- or channel-major within a k-step, 0.1% either way)
// (NT = 2: the activations' second part is zero — the bitboard stem's 0 / 1 inputs — so its
// product w0 x1 would add exact zeros to accumulators that are never -0: left out)
template <int CTW, int PTW, int U0 = 0, int NT = 3>
__device__ __forceinline__ void mma3(f32x4 (&acc)[CTW][PTW], const f16x8 (&a)[PTW][2],
                                     const f16x8 (&w)[CTW][2]) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int c = 0; c < CTW; ++c)
#pragma unroll
            for (int u = U0; u < PTW; ++u)
                acc[c][u] = mfma_h(w[c][t == 1 ? 1 : 0], a[u][t == 2 ? 1 : 0], acc[c][u]);
}

// stem conv 3 -> F as one K = 32 step (27 taps x channels + 5 zeros) on the same tile map
template <int F, int NBOARD, int CTW, int PTW>
__device__ __forceinline__ void stem_h2_load(const uint16_t* __restrict__ blob,
                                             const float* __restrict__ prm, const Layout& L, int NB,
                                             int wave, int lane, EpiH<CTW, PTW>& er,
                                             f16x8 (&w)[CTW][2]) {
    const WaveTilesH<F, CTW, PTW> wt(wave, lane);
    const float* isc = reinterpret_cast<const float*>(blob + h2_scale_off(F, NB));
    load_epi(er, prm + L.stem_b, isc, wt, lane);
    constexpr int CT = F / H2_TM;
    const f16x8* wf = reinterpret_cast<const f16x8*>(blob + h2_stem_off(F, NB)) + wt.ct0 * 64 + lane;
#pragma unroll
    for (int c = 0; c < CTW; ++c)
#pragma unroll
        for (int p = 0; p < 2; ++p) w[c][p] = wf[(p * CT + c) * 64];
}

// the stem's operands are loaded up front (stem_h2_load, with the leaf planes): one global
// round trip before the first MFMA instead of three dependent ones
template <int F, int NBOARD, int CTW, int PTW, int BS, bool ILV>
__device__ __forceinline__ void stem_h2(const float* xin, uint16_t* __restrict__ out,
                                        const f16x8 (&w)[CTW][2], int wave, int lane,
                                        EpiH<CTW, PTW>& er, bool& ovf) {
    const WaveTilesH<F, CTW, PTW> wt(wave, lane, ILV);
    // K order h2_stem_slot: this lane group's taps 2g, 2g + 1 and (groups 0, 1) part of tap 8
    const int kg = lane >> 4, ta = 2 * kg, tb = 2 * kg + 1;
    const int oa = (ta / 3) * 10 + ta % 3, ob = (tb / 3) * 10 + tb % 3;
    const float4* x4 = reinterpret_cast<const float4*>(xin);
    f16x8 a[PTW][2];
#pragma unroll
    for (int u = 0; u < PTW; ++u) {
        using G = GeoH<NBOARD, BS, 64 * CTW * H2_TM / F, ILV>;
        const int px = wt.px[u], b = G::board_of(px), r = G::cell_of(px) / BS,
                  cc = G::cell_of(px) % BS;
        const bool on = px < G::NVALID;               // padding rows: zero input
        const int at = b * 100 + r * 10 + cc;         // tap 0 of this pixel in the padded image
        const float4 z4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        const float4 fa = on ? x4[at + oa] : z4;
        const float4 fb = on ? x4[at + ob] : z4;
        const float4 f8 = on && kg < 2 ? x4[at + 22] : z4;   // tap 8 = (+2 rows, +2 cols)
        const float e6 = kg == 0 ? f8.x : f8.z, e7 = kg == 0 ? f8.y : 0.0f;
        const f32x2 xs[4] = {f32x2{fa.x, fa.y}, f32x2{fa.z, fb.x}, f32x2{fb.y, fb.z},
                             f32x2{e6, e7}};
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        u32x4 h0, h1;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            uint32_t p0, p1;
            split2x2(xs[i], p0, p1);
            h0[i] = p0;
            h1[i] = p1;
        }
        a[u][0] = __builtin_bit_cast(f16x8, h0);
        a[u][1] = __builtin_bit_cast(f16x8, h1);
    }
    f32x4 acc[CTW][PTW];
#pragma unroll
    for (int c = 0; c < CTW; ++c)
#pragma unroll
        for (int u = 0; u < PTW; ++u) acc[c][u] = f32x4{};
    STEM_T(4);
    mma3(acc, a, w);
    {   // wait for the MFMAs (stamp only)
#ifdef RVZ_PHASE_TIMING
        float z = acc[0][0][0];
        asm volatile("" : "+v"(z));
        if (z == 12345.678f) STEM_T(6);
#endif
    }
    STEM_T(5);
    epilogue_h2<F, GeoH<NBOARD, BS, 64 * CTW * H2_TM / F, ILV>::NPIX, CTW, PTW, false, true,
                RVZ_H2_W128 && ILV>(out, acc, er, wt, lane, ovf);
}

// The stem from the leaves' bitboards (the fused self-play kernel: select_phase leaves each
// queued leaf's (P, O, V) = get_canonical_state()'s three planes, mcts.py:582-594, in LDS): the
// same A operands stem_h2 builds from the padded float image (0 / 1 in f16, second part 0; the
// K order of h2_stem_slot), computed from the bits directly.
template <int F, int NBOARD, int CTW, int PTW, int BS, bool ILV>
__device__ __forceinline__ void stem_h2_bits(const uint64_t (&pl)[NBOARD][3],
                                             uint16_t* __restrict__ out, const f16x8 (&w)[CTW][2],
                                             int wave, int lane, EpiH<CTW, PTW>& er, bool& ovf) {
    using G = GeoH<NBOARD, BS, 64 * CTW * H2_TM / F, ILV>;
    typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));
    const WaveTilesH<F, CTW, PTW> wt(wave, lane, ILV);
    const int kg = lane >> 4, ta = 2 * kg, tb = 2 * kg + 1;
    f16x8 a[PTW][2];
#pragma unroll
    for (int u = 0; u < PTW; ++u) {
        const int px = wt.px[u], b = G::board_of(px), cell = G::cell_of(px);
        const int r = cell / BS, c = cell % BS;
        const bool on = px < G::NVALID;
        uint64_t P = pl[0][0], O = pl[0][1], V = pl[0][2];
#pragma unroll
        for (int k = 1; k < NBOARD; ++k)
            if (b == k) {
                P = pl[k][0];
                O = pl[k][1];
                V = pl[k][2];
            }
        auto bit = [&](int t, uint64_t plane) -> uint16_t {
            const int rr = r + t / 3 - 1, cc = c + t % 3 - 1;
            const bool in = on && (unsigned)rr < (unsigned)BS && (unsigned)cc < (unsigned)BS;
            return in && ((plane >> (rr * BS + cc)) & 1ull) ? (uint16_t)0x3C00 : (uint16_t)0;
        };
        u16x8 h;
        h[0] = bit(ta, P);
        h[1] = bit(ta, O);
        h[2] = bit(ta, V);
        h[3] = bit(tb, P);
        h[4] = bit(tb, O);
        h[5] = bit(tb, V);
        h[6] = kg == 0 ? bit(8, P) : (kg == 1 ? bit(8, V) : (uint16_t)0);
        h[7] = kg == 0 ? bit(8, O) : (uint16_t)0;
        a[u][0] = __builtin_bit_cast(f16x8, h);
        a[u][1] = f16x8{};
    }
    f32x4 acc[CTW][PTW];
#pragma unroll
    for (int c = 0; c < CTW; ++c)
#pragma unroll
        for (int u = 0; u < PTW; ++u) acc[c][u] = f32x4{};
    mma3<CTW, PTW, 0, 2>(acc, a, w);
    epilogue_h2<F, G::NPIX, CTW, PTW, false, true, RVZ_H2_W128 && ILV>(out, acc, er, wt, lane, ovf);
}

template <int F, int NBOARD, int CTW, int PTW, bool RES, int BS, bool ILV, int GRP = 0,
          bool LASTH = false, class K = H2Def>
__device__ __forceinline__ void conv_h2(const uint16_t* __restrict__ in, uint16_t* __restrict__ out,
                                        const H2W& wr, int wl,   // layer base, f16x8 units
                                        const float* __restrict__ bias,
                                        const float* __restrict__ isc, int wave, int lane,
                                        f16x8 (&bc)[K::PD][CTW][2], EpiH<CTW, PTW>& er,
                                        bool& ovf, HeadPart hp = HeadPart{}) {
    using G = GeoH<NBOARD, BS, 64 * CTW * H2_TM / F, ILV>;
    using C = CfgH<F, G::NPIX>;
    constexpr int KS = C::KS, CT = C::CT, NIT = C::NIT, PD = K::PD, APD = K::APD;
    // ILV: tile 0 is board row 0 (pixel group 0) or row 7 (group 1), and the taps with dr = -1
    // (row 0) or dr = +1 (row 7) leave the boards for all its pixels: tile 0's A loads and MFMAs
    // are skipped in those k-steps (1/12 of the conv MFMAs).
    // RVZ_H2_MIRROR 0 (default, NAT): both groups walk the taps in natural order, so the two waves
    // of a channel group fetch the same weight fragments at about the same time (L1 hits), and
    // each skips in its own window, group 0 in [0, 3 KS) (dr = -1), group 1 in [6 KS, 9 KS)
    // (dr = +1), both compile-time: the kernel instantiates the whole trunk once per group (GRP)
    // behind one wave-uniform branch (190 VGPRs; the same choice made per layer needed 224, per
    // k-step 248). Whole-bench A/B, one box: +2.8% over the row mirror
    // (profiles/r02ah_ab_nat.txt).
    // RVZ_H2_MIRROR 2 (row mirror): group 1 walks the tap rows in reverse (dr -> -dr) so both
    // groups skip in k-steps [0, 3 KS) and share fragments only in the middle tap row: -3.2%
    // trunk against no skip (profiles/r02k_ab_h2_mirror_c2.json); 1 (full mirror) shares only
    // the centre tap: -2.1%.
    constexpr bool NAT = ILV && RVZ_H2_MIRROR == 0;
    const WaveTilesH<F, CTW, PTW> wt(wave, lane, ILV);
    const bool mirror = ILV && !NAT && wave / WaveTilesH<F, CTW, PTW>::CG != 0;
    // is tile 0 skipped in k-step i (compile-time once the k-loop is unrolled)
    auto skip0 = [](int i) -> bool {
        if (!ILV) return false;
        if (NAT) return GRP == 0 ? i < 3 * KS : (i >= 6 * KS && i < 9 * KS);
        return i < 3 * KS;
    };
    if constexpr (!K::LATE) load_epi(er, bias, isc, wt, lane);   // lands during the k-loop
    const int kq = lane >> 4;                         // this lane's 8-channel slot in a k-step
    unsigned pmask[PTW];                              // valid taps in iteration order
#pragma unroll
    for (int u = 0; u < PTW; ++u) {
        const unsigned m = G::taps(wt.px[u]);
        pmask[u] = !mirror ? m
                   : RVZ_H2_MIRROR == 1 ? __builtin_bitreverse32(m) >> 23
                                        : ((m & 7u) << 6) | (m & 0x38u) | ((m >> 6) & 7u);
    }
    f32x4 acc[CTW][PTW];
#pragma unroll
    for (int c = 0; c < CTW; ++c)
#pragma unroll
        for (int u = 0; u < PTW; ++u) acc[c][u] = f32x4{};
    const int wu = wl + wt.ct0 * 64;
    auto load_b = [&](f16x8 (&bq)[CTW][2], int it) {
        const int f = wu + h2_frag<F>(it, mirror);
#pragma unroll
        for (int c = 0; c < CTW; ++c)
#pragma unroll
            for (int p = 0; p < 2; ++p) bq[c][p] = wr.load(f + (p * CT + c) * 64, lane);
    };
    auto load_a = [&](f16x8 (&aq)[PTW][2], int it) {
        const int t = it / KS, ks = it - t * KS;
        const int off = mirror ? G::tap_offset(h2_mirror_tap(t)) : G::tap_offset(t);
#pragma unroll
        for (int u = (skip0(it) ? 1 : 0); u < PTW; ++u) {
            const int nat = wt.px[u] + off;
            const int row = (pmask[u] >> t) & 1u ? nat : C::ZROW + (nat & 7);
            const uint16_t* ap = in + C::at(row, 0, kq) + ks * C::KSP;
#pragma unroll
            for (int p = 0; p < 2; ++p)
                aq[u][p] = *reinterpret_cast<const f16x8*>(ap + p * C::PLANE);
        }
    };
    f16x8 bq[NIT + PD][CTW][2];
    f16x8 aq[APD + 1][PTW][2];
#pragma unroll
    for (int d = 0; d < PD; ++d)
#pragma unroll
        for (int c = 0; c < CTW; ++c)
#pragma unroll
            for (int p = 0; p < 2; ++p) bq[d][c][p] = bc[d][c][p];
#pragma unroll
    for (int d = 0; d < APD; ++d) load_a(aq[d], d);
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
        const int ia = it + APD;                      // the A operands loaded this k-step
        if (ia < NIT) load_a(aq[ia % (APD + 1)], ia);
        load_b(bq[it + PD], it + PD);
        const bool sa = ia < NIT && skip0(ia);        // next A load without tile 0
        if (skip0(it)) {
            mma3<CTW, PTW, 1>(acc, aq[it % (APD + 1)], bq[it]);
            if (sa) interleave_loads<0, 3 * CTW * (PTW - 1), 2 * (PTW - 1), 2 * CTW>();
            else interleave_loads<0, 3 * CTW * (PTW - 1), 2 * PTW, 2 * CTW>();
        } else {
            mma3(acc, aq[it % (APD + 1)], bq[it]);
            if (sa) interleave_loads<0, 3 * CTW * PTW, 2 * (PTW - 1), 2 * CTW>();
            else interleave_loads<0, 3 * CTW * PTW, 2 * PTW, 2 * CTW>();
        }
        __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int d = 0; d < PD; ++d)
#pragma unroll
        for (int c = 0; c < CTW; ++c)
#pragma unroll
            for (int p = 0; p < 2; ++p) bc[d][c][p] = bq[NIT + d][c][p];
    if constexpr (K::LATE) load_epi(er, bias, isc, wt, lane);
    // conv A (block input -> t): the skip input stays in er.res; conv B adds it and keeps
    if constexpr (LASTH) {
        f32x4 hw[3][CTW];                             // the head convs' weights (L2, once)
#pragma unroll
        for (int c = 0; c < CTW; ++c) {
            const int n = (wt.ct0 + c) * H2_TM + 4 * (lane >> 4);
            hw[0][c] = *reinterpret_cast<const f32x4*>(hp.pol + n);
            hw[1][c] = *reinterpret_cast<const f32x4*>(hp.pol + F + n);
            hw[2][c] = *reinterpret_cast<const f32x4*>(hp.val + n);
        }
        epilogue_heads<F, G::NPIX, CTW, PTW>(acc, er, wt, wave, lane, hw, hp.part, ovf);
    } else
        epilogue_h2<F, G::NPIX, CTW, PTW, RES, RES, RVZ_H2_W128 && ILV, K::SKIP>(out, acc, er,
                                                                                  wt, lane, ovf);
}

// the leaf planes of NBOARD boards -> the halo-padded stem input xin[b][10x10][4] (halo and, for
// BS < 8, the unused rows/columns 0), staged through registers: the loads are issued with the
// stem's weight loads, before anything waits
template <int NBOARD, int BS, int NTHR>
struct XinStage {
    static constexpr int N = NBOARD * 100 * 4, PER = (N + NTHR - 1) / NTHR;
    float v[PER];
    // board b's planes are row gb[b] of x (gb[b] < 0: no board, zero input)
    __device__ void load(const float* __restrict__ x, const int (&gb)[NBOARD], int tid) {
        constexpr int CELLS = BS * BS;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int i = tid + j * NTHR;
            const int b = i / 400, rem = i % 400, p10 = rem >> 2, ch = rem & 3;
            const int r = p10 / 10 - 1, c = p10 % 10 - 1;
            int g = gb[0];
#pragma unroll
            for (int k = 1; k < NBOARD; ++k) g = b == k ? gb[k] : g;
            const bool in = i < N && ch < 3 && (unsigned)r < (unsigned)BS &&
                            (unsigned)c < (unsigned)BS && g >= 0;
            v[j] = in ? x[((size_t)g * 3 + ch) * CELLS + r * BS + c] : 0.0f;
        }
    }
    __device__ void store(float* xin, int tid) const {
#pragma unroll
        for (int j = 0; j < PER; ++j)
            if (tid + j * NTHR < N) xin[tid + j * NTHR] = v[j];
    }
};

// hpv rows in a global workspace, board b at row gb[b] (< 0: not stored)
template <int NBOARD>
struct HeadsGlobalIdx {
    float* p;
    int gb[NBOARD];
    __device__ HeadsGlobalIdx(float* p_, const int (&g)[NBOARD]) : p(p_) {
#pragma unroll
        for (int k = 0; k < NBOARD; ++k) gb[k] = g[k];
    }
    __device__ void store(int b, int i, float v) const {
        int g = gb[0];
#pragma unroll
        for (int k = 1; k < NBOARD; ++k) g = b == k ? gb[k] : g;
        if (g >= 0) p[(size_t)g * 192 + i] = v;
    }
};

// hpv rows straight into the FC heads' LDS input (heads_fc16 with its rows in place): board b
// is column slot0 + b (< 0 slots: not stored); policy planes at [0, 2 cells), the value plane at
// PK (the heads' row layout; 8x8: no gaps)
template <int BS>
struct HeadsInLds {
    float* in;
    int slot0, nslots;
    __device__ void store(int b, int i, float v) const {
        constexpr int CELLS = BS * BS, PIN = 2 * CELLS, PK = (PIN + 15) / 16 * 16;
        constexpr int ROW = heads_in_floats(BS) / 16;
        const int sl = slot0 + b;
        if (sl < nslots) in[sl * ROW + (i < PIN ? i : PK + (i - PIN))] = v;
    }
};

// One pass of the workgroup (256 threads) over NBOARD boards: board b's leaf planes are row gb[b]
// of x ([rows][3][BS*BS], gb[b] < 0: no board), its 1x1 head-conv outputs go to row gb[b] of
// work ([rows][192]: policy planes, then the value plane). smem: CfgH<..>::BYTES of LDS, free on
// entry and on return. ovf |= an activation overflowed f16 (the caller's sticky word).
// Input of a pass: board b's leaf planes are row gb[b] of x (float [rows][3][BS*BS]), or, when
// bits is set, the bitboards bits[3 * b .. 3 * b + 2] = (P, O, V) (LDS). Output: the 1x1
// head-conv rows through hout (HeadsGlobalIdx: row gb[b] of work; HeadsInLds: the FC heads' LDS
// input rows).
struct NoHook {
    __device__ __forceinline__ void operator()() const {}
};
template <int F, int NBOARD, int CTW, int PTW, int BS, class HOut, class K = H2Def,
          class Bar = BarWG, class Hook = NoHook>
__device__ __forceinline__ void h2_pass(char* smem, const float* __restrict__ x,
                                        const int (&gbv)[NBOARD], const uint64_t* bits,
                                        const float* __restrict__ prm, const Layout& L,
                                        const uint16_t* __restrict__ blob, int n_blocks,
                                        const HOut& hout, int tid, int lane, int wave, bool& ovf,
                                        const Bar& bar = Bar{}, const Hook& hook = Hook{}) {
    using WT = WaveTilesH<F, CTW, PTW>;
    constexpr bool ILV = RVZ_H2_ILV && NBOARD == 2 && BS == 8 && PTW == 4 && WT::CG == 2;
    using G = GeoH<NBOARD, BS, 64 * CTW * H2_TM / F, ILV>;
    using C = CfgH<F, G::NPIX>;
    constexpr int NTHR = 256;
    uint16_t* actA = reinterpret_cast<uint16_t*>(smem);
    uint16_t* actB = actA + C::ACT;
    float* xin = reinterpret_cast<float*>(actB);     // free until the first conv writes B
    int gb[NBOARD];                                   // workgroup-uniform: scalar registers
#pragma unroll
    for (int k = 0; k < NBOARD; ++k) gb[k] = __builtin_amdgcn_readfirstlane(gbv[k]);

    PASS_NOW(tp0);
    // zero rows of both buffers, both parts, every k-step plane (4 * KS planes of KSP)
    for (int i = tid; i < 4 * C::KS * 8 * H2_K; i += NTHR) {
        const int plane = i / (8 * H2_K), k = i % (8 * H2_K);
        actA[plane * C::KSP + C::ZROW * H2_K + k] = 0;
    }
    // (issuing the stem's loads before the first conv's weight prefetch measured neutral: the
    // stem's epilogue time is the partner workgroup's MFMAs sharing the SIMD, not a load wait)
    const H2W wr(blob, h2_blob_elems(F, n_blocks));
    // from the weight prefetch to the last residual block; NAT (RVZ_H2_MIRROR 0): one instance
    // per pixel group (its own tile-0 skip window), chosen by a wave-uniform branch
    const bool grp1 = ILV && RVZ_H2_MIRROR == 0 && wave / WT::CG != 0;
    constexpr bool HEPI = RVZ_H2_HEADS_EPI && !K::SKIP && ILV;   // C2 shape (F = 128 spilled)
    auto trunk = [&](auto grp) {
        constexpr int GR = decltype(grp)::value;
        f16x8 bc[K::PD][CTW][2];
        if (n_blocks > 0) {
            const int wu = WT(wave, lane).ct0 * 64;
            const bool mirror = ILV && RVZ_H2_MIRROR != 0 && wave / WT::CG != 0;   // as conv_h2
#pragma unroll
            for (int s = 0; s < K::PD; ++s) {
                const int f = wu + h2_frag<F>(s, mirror);
#pragma unroll
                for (int c = 0; c < CTW; ++c)
#pragma unroll
                    for (int p = 0; p < 2; ++p) bc[s][c][p] = wr.load(f + (p * C::CT + c) * 64, lane);
            }
        }
        EpiH<CTW, PTW> er;
        f16x8 ws[CTW][2];
        if (bits) {   // leaf bitboards in LDS: no global round trip, no padded image
            uint64_t pl[NBOARD][3];
#pragma unroll
            for (int b = 0; b < NBOARD; ++b)
#pragma unroll
                for (int ch = 0; ch < 3; ++ch) {
                    const uint64_t v = bits[3 * b + ch];
                    pl[b][ch] = ((uint64_t)__builtin_amdgcn_readfirstlane((int)(v >> 32)) << 32) |
                                (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
                }
            stem_h2_load<F, NBOARD, CTW, PTW>(blob, prm, L, n_blocks, wave, lane, er, ws);
            stem_h2_bits<F, NBOARD, CTW, PTW, BS, ILV>(pl, actA, ws, wave, lane, er, ovf);
        } else {
            XinStage<NBOARD, BS, NTHR> st;
            st.load(x, gb, tid);
            stem_h2_load<F, NBOARD, CTW, PTW>(blob, prm, L, n_blocks, wave, lane, er, ws);
            STEM_T(0);
            st.store(xin, tid);
            STEM_T(1);
            bar();
            STEM_T(2);
            stem_h2<F, NBOARD, CTW, PTW, BS, ILV>(xin, actA, ws, wave, lane, er, ovf);
            STEM_T(3);
        }
        bar();
        PHASE(1);
        {
            PASS_NOW(tp1);
            PASS_ADD(0, tp1 - tp0);
        }
        const int64_t LW = h2_layer_elems(F);
        const float* isc = reinterpret_cast<const float*>(blob + h2_scale_off(F, n_blocks)) + F;
        for (int blk = 0; blk < n_blocks - (HEPI ? 1 : 0); ++blk) {
            const int l1 = 2 * blk, l2 = 2 * blk + 1;
            conv_h2<F, NBOARD, CTW, PTW, false, BS, ILV, GR, false, K>(actA, actB, wr, (int)(l1 * LW / 8),
                                                          prm + L.res_b + (size_t)l1 * F,
                                                          isc + l1 * F, wave, lane, bc, er, ovf);
            if (blk == 0) PHASE(5);
            bar();
            if (blk == 0) PHASE(6);
            conv_h2<F, NBOARD, CTW, PTW, true, BS, ILV, GR, false, K>(actB, actA, wr, (int)(l2 * LW / 8),
                                                         prm + L.res_b + (size_t)l2 * F,
                                                         isc + l2 * F, wave, lane, bc, er, ovf);
            bar();
        }
        if (HEPI && n_blocks > 0) {   // the last block: its conv B ends in the head convs
            const int l1 = 2 * n_blocks - 2, l2 = 2 * n_blocks - 1;
            conv_h2<F, NBOARD, CTW, PTW, false, BS, ILV, GR, false, K>(actA, actB, wr, (int)(l1 * LW / 8),
                                                          prm + L.res_b + (size_t)l1 * F,
                                                          isc + l1 * F, wave, lane, bc, er, ovf);
            bar();
            conv_h2<F, NBOARD, CTW, PTW, true, BS, ILV, GR, true, K>(
                actB, actA, wr, (int)(l2 * LW / 8), prm + L.res_b + (size_t)l2 * F, isc + l2 * F,
                wave, lane, bc, er, ovf,
                HeadPart{prm + L.pol_w, prm + L.val_w, reinterpret_cast<float*>(actA)});
            bar();
        }
    };
    if (grp1)
        trunk(std::integral_constant<int, 1>{});
    else
        trunk(std::integral_constant<int, 0>{});
    PHASE(2);
    PASS_NOW(tp2);
    PASS_ADD(1, tp2 - tp0);   // stem + tower
    hook();                   // the caller's loads that may land during the head convs
    // the 1x1 head convs -> work (the FC heads are the next launch, k_heads_mfma)
    if (HEPI && n_blocks > 0) {   // the channel-group partials of the last epilogue, + bias, ReLU
        constexpr int CELLS = BS * BS, CG = WT::CG;
        const float* part = reinterpret_cast<const float*>(actA);
        const HOut& hpv = hout;
        for (int o = tid; o < NBOARD * 3 * CELLS; o += NTHR) {
            const int c2 = o / (NBOARD * CELLS), rem = o % (NBOARD * CELLS);
            const int b = rem / CELLS, cell = rem % CELLS;
            const int px = G::row_of(b, cell);
            float acc = 0.0f;
#pragma unroll
            for (int g = 0; g < CG; ++g) acc += part[(g * 3 + c2) * G::NPIX + px];
            const float bias = c2 < 2 ? prm[L.pol_b + c2] : prm[L.val_b];
            hpv.store(b, c2 * CELLS + cell, fmaxf(acc + bias, 0.0f));
        }
    } else {
        head_convs<F, NBOARD, NTHR, BS, true, ILV>(ActH2<F, G::NPIX>{actA},
                                                  reinterpret_cast<float*>(actB), prm, L, hout,
                                                  tid, bar);
    }
#ifdef RVZ_PLAY_TIMING
    {
        PASS_NOW(tp3);
        PASS_ADD(2, tp3 - tp2);
        PASS_ADD(3, 1);
    }
#endif
}

// RVZ_H2_MAXV (experiments): cap the trunk's VGPRs so that a k_step wave (80) fits on a SIMD
// beside two trunk waves (2 x 216 + 80 = 512)
#ifdef RVZ_H2_MAXV
#define RVZ_H2_VGPR_ATTR __attribute__((amdgpu_num_vgpr(RVZ_H2_MAXV)))
#else
#define RVZ_H2_VGPR_ATTR
#endif
// bits 52-55 of a workgroup's end stamp: the XCD it ran on (HW_REG_XCC_ID; bench.py --stamps-dump)
__device__ __forceinline__ uint64_t stamp_xcc() {
    return (uint64_t)(__builtin_amdgcn_s_getreg((31 << 11) | 20) & 0xF) << 52;
}
}  // namespace
