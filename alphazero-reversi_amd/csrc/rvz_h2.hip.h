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
//   [activation ranges: float[1 + 2*NB][2] {K, Bb} (h2_range_off; the activation range section below)]

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2v __attribute__((ext_vector_type(2)));

#ifndef RVZ_H2_PD
#define RVZ_H2_PD 2          // weight prefetch distance, k-steps
#endif
#ifndef RVZ_H2_APD
#define RVZ_H2_APD 1         // activation prefetch distance, k-steps
#endif
#ifndef RVZ_H2_PD256
#define RVZ_H2_PD256 1       // F = 256 (one workgroup per CU): weight prefetch distance, k-steps
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
// zero k-steps after the last layer: the weight prefetch of the next (absent) layer reads them
__host__ __device__ inline int64_t h2_pad_ksteps(int) { return 4; }
static_assert(RVZ_H2_PD <= 4 && RVZ_H2_PD256 <= 4, "prefetch stays inside the padded blob");
__host__ __device__ inline int64_t h2_stem_off(int F, int NB) {
    return 2 * NB * h2_layer_elems(F) + h2_pad_ksteps(F) * h2_kstep_elems(F);
}
__host__ __device__ inline int64_t h2_scale_off(int F, int NB) {   // uint16 units, 16-B aligned
    return h2_stem_off(F, NB) + (int64_t)2 * F * H2_K;
}
// the activation-range table (uint16 units, 16-B aligned): float[1 + 2 NB][2] = per layer (stem,
// then the trunk convs) {K = max over output channels of sum |w| (BN-folded, unscaled), Bb = max
// |bias|}: a layer's outputs are bounded by K * max|input| + Bb (+ the skip input's max)
__host__ __device__ inline int64_t h2_range_off(int F, int NB) {
    return h2_scale_off(F, NB) + (int64_t)2 * (1 + 2 * NB) * F;
}
__host__ __device__ inline int64_t h2_blob_elems(int F, int NB) {
    return h2_range_off(F, NB) + ((int64_t)4 * (1 + 2 * NB) + 7) / 8 * 8;
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
    static constexpr int NBRD = NB;
    static constexpr bool ILVD = ILV;
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
    static constexpr int RMAX = 2 * ACT * 2;         // byte offset of the range maxima (RangeLds)
    static constexpr int BYTES = RMAX + 3 * 4 * 4 * 4 + 16;  // + the pass's overflow word
    static constexpr int NIT = 9 * KS;
    static constexpr int CT = F / H2_TM;
    static_assert((PLANE * 2) % 16 == 0 && (KSP * 2) % 16 == 0, "16-byte aligned planes");
    static_assert(BYTES <= 160 * 1024, "fits the LDS of a CU");
    // halves offset of (row, k-step plane ks, 8-channel slot q in 0..3)
    static __device__ __forceinline__ int at(int row, int ks, int q) {
        return ks * KSP + row * H2_K + 8 * (q ^ ((row >> 1) & 3));
    }
};

// ---- activation range ------------------------------------------------
// The f16 parts of an activation overflow at 65520. Each board's image is therefore stored as
// x * 2^-s, with s chosen per board and layer, before the layer's epilogue writes it, from a
// bound on the layer's outputs: K * (the measured max of its input image) + Bb (+ the max of
// the skip input), K = max over output channels of sum |w| and Bb = max |bias| from the blob's
// range table (rvz_resnet_h2_weights). s = 0 while the bound stays below 2^15 — every random-init
// and trained net measured — and then the stored image, the MFMAs and every output are bitwise
// those of the unscaled kernel (the scaled path is a separate, wave-uniform branch). A scaled
// board keeps fp32-class accuracy relative to its largest activation; values below 2^(s - 3)
// lose low-order bits to f16 subnormals. The next layer's epilogue multiplies its accumulator by
// 2^s (exact) before the bias. Maxima: each wave's per-board max of its true (unscaled) outputs
// goes to LDS (RangeLds), where the next layer reads it after the barrier between the two.
__device__ __forceinline__ int range_exp(float bound) {
    if (!(bound < 0x1p100f)) return 100;             // inf / NaN weights: the image is lost anyway
    int e = 0;
    (void)frexpf(bound, &e);                         // bound < 2^e
    return e > 15 ? e - 15 : 0;
}
__device__ __forceinline__ float pow2f(int s) {      // 2^s, |s| <= 126
    return __int_as_float((127 + s) << 23);
}
// the max of a non-negative value over the wave, wave-uniform: DPP within rows of 16 lanes
// (quad swaps, then row shifts by 4 and 8 with zero fill), then the four row maxima
__device__ __forceinline__ float wave_max_nonneg(float v) {
    auto up = [](float x, auto ctrl) {
        return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x),
                                                          decltype(ctrl)::value, 0xF, 0xF, true));
    };
    v = fmaxf(v, up(v, std::integral_constant<int, 0xB1>{}));    // quad_perm [1, 0, 3, 2]
    v = fmaxf(v, up(v, std::integral_constant<int, 0x4E>{}));    // quad_perm [2, 3, 0, 1]
    v = fmaxf(v, up(v, std::integral_constant<int, 0x114>{}));   // row_shr:4
    v = fmaxf(v, up(v, std::integral_constant<int, 0x118>{}));   // row_shr:8: lane 15 of a row
    auto rl = [&](int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); };
    return fmaxf(fmaxf(rl(15), rl(31)), fmaxf(rl(47), rl(63)));
}
template <int NB>
struct RangeS {                     // wave-uniform scale exponents of an image, 8 bits per board
    int pk = 0;
    __device__ int s(int k) const { return (pk >> (8 * k)) & 0xFF; }
    __device__ bool any() const { return pk != 0; }
    // 2^(sign * s(b)) for a lane's board b (b >= NB: padding rows, 1)
    __device__ float mul(int b, int sign) const {
        return b < NB ? pow2f(sign * ((pk >> (8 * b)) & 0xFF)) : 1.0f;
    }
};
// maxima in LDS: [slot][board < 4][wave < 4] floats at CfgH::RMAX; slots 0 / 2 = the inputs of
// even / odd residual blocks (the stem and conv B write them), 1 = conv A's outputs (and the
// stem's input in the pull-style pass)
struct RangeLds {
    float* p;
    __device__ float* slot(int par) const { return p + par * 16; }
    // a wave's overflow word of the pass (bit b: board b stored a value past f16's range,
    // unranged mode): one per wave, so each wave clears and sets its own in program order
    __device__ unsigned* ovw(int wave) const { return reinterpret_cast<unsigned*>(p + 48) + wave; }
    // the pass's overflow bits: every wave's word (after a barrier that follows their epilogues)
    __device__ unsigned ov_all() const {
        const unsigned* q = reinterpret_cast<const unsigned*>(p + 48);
        return (unsigned)__builtin_amdgcn_readfirstlane((int)(q[0] | q[1] | q[2] | q[3]));
    }
    // the max over the 4 waves of board b (wave-uniform)
    __device__ float read(int par, int b) const {
        const float* q = slot(par) + 4 * b;
        const float m = fmaxf(fmaxf(q[0], q[1]), fmaxf(q[2], q[3]));
        return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__float_as_int(m)));
    }
};
// the output scale exponents of a layer from its bound, per board
template <int NB>
__device__ __forceinline__ RangeS<NB> range_out(const float (&m_in)[NB], float K, float Bb,
                                               const float* m_skip) {
    RangeS<NB> r;
#pragma unroll
    for (int k = 0; k < NB; ++k) {
        // (a separate multiply and add: an fma of two scalar operands here miscompiles on
        // gfx950, ROCm 7.2 — "VOP* instruction violates constant bus restriction")
        float b = K * m_in[k] + Bb + (m_skip ? m_skip[k] : 0.0f);
        r.pk |= range_exp(b * 1.001f) << (8 * k);    // margin for the fp32 rounding of the sums
    }
    r.pk = __builtin_amdgcn_readfirstlane(r.pk);
    return r;
}

// activation reader for the heads (join of the two parts, times the board's scale 2^s)
template <int F, int NPIX>
struct ActH2 {
    const uint16_t* p;
    int pk = 0;                                      // the image's RangeS exponents
    __device__ float mul(int b) const { return pow2f((pk >> (8 * b)) & 0xFF); }
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
// lane's 16-byte slot the only VGPR.
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
// [tap][kstep][part][ctile][lane]
template <int F>
__device__ __forceinline__ int h2_frag(int it) {
    constexpr int KS = F / H2_K, NIT = 9 * KS, CT = F / H2_TM, KSTEP = 2 * CT * 64;
    const int lay = it / NIT, itn = it % NIT, t = itn / KS, ks = itn % KS;
    return (lay * NIT + t * KS + ks) * KSTEP;
}

// The skip input of a residual block stays in fp32 registers (EpiH::res) from conv A's epilogue
// to conv B's. (Re-reading it from LDS as its two parts let a k_step or FC-heads wave share a SIMD
// with two trunk waves under an earlier tap order; under the natural-order trunk the registers
// win: +1.05% per ply, profiles/r02ap_ab_skipreg.txt.) Rejected epilogue / knob variants are
// kept as patches in tools/patches/ (README there).
template <int CTW, int PTW>
struct EpiH {
    f32x4 bias[CTW], isc[CTW];       // per out-channel bias, inverse weight scale
    float res[CTW][PTW][4];          // the block input (fp32) of this lane's outputs
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
// channels of one pixel per tile -> two 8-byte writes.
// Activation range (the section above), two modes. RANGED false (every pass first): the values are
// stored unscaled, and a board with a value past f16's range sets its bit in the pass's overflow
// word *ovw (LDS; a wave-uniform test, one compare per value as the sticky flag always cost).
// RANGED true (only a pass whose word is set, re-run for those boards): the accumulator is
// multiplied by 2^sin[b] and the stored value by 2^-sout[b] (the scaled branch, wave-uniform),
// and the per-board max of the true outputs goes to rm_out[b][wave] (lane 0) for the next
// layer's bound; a stored max past f16's range would be a bound error (the sticky word ovf).
template <int F, int NPIX, int CTW, int PTW, bool RES, bool KEEP, class G>
__device__ __forceinline__ void epilogue_h2(uint16_t* __restrict__ out,
                                            const f32x4 (&acc)[CTW][PTW], EpiH<CTW, PTW>& er,
                                            const WaveTilesH<F, CTW, PTW>& wt, int lane, int wave,
                                            bool& ovf, bool rg, const RangeS<G::NBRD>& sin,
                                            const RangeS<G::NBRD>& sout, float* rm_out,
                                            unsigned* ovw) {
    using C = CfgH<F, NPIX>;
    constexpr int NB = G::NBRD;
    // LB: a lane's pixels all belong to one board (ILV: board = pixel column group; NB = 1), so
    // one running max / overflow flag and one pair of multipliers per lane; else (packed 6x6)
    // per board (max) or per tile (flag)
    constexpr bool LB = G::ILVD || NB == 1;
    constexpr int NM = LB ? 1 : NB;
    constexpr int NO = LB ? 1 : PTW;
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    float mt[NM];                                    // max of this lane's outputs (ranged)
    bool oflow[NO];                                  // a value past f16's range (not ranged)
#pragma unroll
    for (int u = 0; u < NM; ++u) mt[u] = 0.0f;
#pragma unroll
    for (int u = 0; u < NO; ++u) oflow[u] = false;
    auto body = [&](auto scaled, auto ranged) {
        constexpr bool SC = decltype(scaled)::value, RANGED = decltype(ranged)::value;
        float mi0 = 1.0f, mo0 = 1.0f;
        if constexpr (SC && LB) {
            mi0 = sin.mul(G::board_of(wt.px[0]), 1);
            mo0 = sout.mul(G::board_of(wt.px[0]), -1);
        }
#pragma unroll
        for (int c = 0; c < CTW; ++c)
#pragma unroll
            for (int u = 0; u < PTW; ++u) {
                const int n0 = (wt.ct0 + c) * H2_TM + 4 * (lane >> 4);
                const int o = C::at(wt.px[u], n0 / H2_K, (n0 % H2_K) >> 3) + (n0 & 4);
                float mi = mi0, mo = mo0;
                if constexpr (SC && !LB) {
                    mi = sin.mul(G::board_of(wt.px[u]), 1);
                    mo = sout.mul(G::board_of(wt.px[u]), -1);
                }
                u32x2 d0, d1;
#pragma unroll
                for (int hf = 0; hf < 2; ++hf) {
                    f32x2 v;
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        const int j = 2 * hf + e;
                        float x = fmaf(SC ? acc[c][u][j] * mi : acc[c][u][j], er.isc[c][j],
                                       er.bias[c][j]);
                        if (RES) x += er.res[c][u][j];
                        x = fmaxf(x, 0.0f);
                        if constexpr (!RANGED) {
                            oflow[LB ? 0 : u] |= x >= 65520.0f;
                        } else if constexpr (LB) {
                            mt[0] = fmaxf(mt[0], x);
                        } else {
                            const int bu = G::board_of(wt.px[u]);
#pragma unroll
                            for (int k = 0; k < NB; ++k) mt[k] = bu == k ? fmaxf(mt[k], x) : mt[k];
                        }
                        if constexpr (KEEP) er.res[c][u][j] = x;
                        v[e] = SC ? x * mo : x;
                    }
                    uint32_t h0, h1;
                    split2x2(v, h0, h1);
                    d0[hf] = h0;
                    d1[hf] = h1;
                }
                *reinterpret_cast<u32x2*>(out + o) = d0;
                *reinterpret_cast<u32x2*>(out + C::PLANE + o) = d1;
            }
    };
    if (!rg) {
        body(std::false_type{}, std::false_type{});
        bool any = false;
#pragma unroll
        for (int u = 0; u < NO; ++u) any |= oflow[u];
        if (__builtin_amdgcn_ballot_w64(any) != 0ull) {      // rare: which boards
            unsigned bits = 0;
#pragma unroll
            for (int u = 0; u < NO; ++u)
#pragma unroll
                for (int k = 0; k < NB; ++k)
                    if (__builtin_amdgcn_ballot_w64(oflow[u] && G::board_of(wt.px[u]) == k))
                        bits |= 1u << k;
            if (lane == 0) atomicOr(ovw, bits);
        }
        return;
    } else {
        if (sin.any() || sout.any())
            body(std::true_type{}, std::true_type{});
        else
            body(std::false_type{}, std::true_type{});
#pragma unroll
        for (int k = 0; k < NB; ++k) {
            float m = LB ? (G::board_of(wt.px[0]) == k ? mt[0] : 0.0f) : mt[k];
            m = wave_max_nonneg(m);
            ovf |= m * pow2f(-sout.s(k)) >= 65520.0f;
            if (lane == 0) rm_out[4 * k + wave] = m;
        }
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
                                        EpiH<CTW, PTW>& er, bool& ovf, bool rg,
                                        const RangeS<NBOARD>& sout, float* rm_out,
                                        unsigned* ovw) {
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
    using G = GeoH<NBOARD, BS, 64 * CTW * H2_TM / F, ILV>;
    epilogue_h2<F, G::NPIX, CTW, PTW, false, true, G>(out, acc, er, wt, lane, wave, ovf, rg,
                                                      RangeS<NBOARD>{}, sout, rm_out, ovw);
}

// The stem from the leaves' bitboards (the fused self-play kernel: select_phase leaves each
// queued leaf's (P, O, V) = get_canonical_state()'s three planes, mcts.py:582-594, in LDS): the
// same A operands stem_h2 builds from the padded float image (0 / 1 in f16, second part 0; the
// K order of h2_stem_slot), computed from the bits directly.
template <int F, int NBOARD, int CTW, int PTW, int BS, bool ILV>
__device__ __forceinline__ void stem_h2_bits(const uint64_t (&pl)[NBOARD][3],
                                             uint16_t* __restrict__ out, const f16x8 (&w)[CTW][2],
                                             int wave, int lane, EpiH<CTW, PTW>& er, bool& ovf,
                                             bool rg,
                                             const RangeS<NBOARD>& sout, float* rm_out,
                                             unsigned* ovw) {
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
    epilogue_h2<F, G::NPIX, CTW, PTW, false, true, G>(out, acc, er, wt, lane, wave, ovf, rg,
                                                      RangeS<NBOARD>{}, sout, rm_out, ovw);
}

template <int F, int NBOARD, int CTW, int PTW, bool RES, int BS, bool ILV, int GRP,
          int PD = RVZ_H2_PD, int APD = RVZ_H2_APD>
__device__ __forceinline__ void conv_h2(const uint16_t* __restrict__ in, uint16_t* __restrict__ out,
                                        const H2W& wr, int wl,   // layer base, f16x8 units
                                        const float* __restrict__ bias,
                                        const float* __restrict__ isc, int wave, int lane,
                                        f16x8 (&bc)[PD][CTW][2], EpiH<CTW, PTW>& er,
                                        bool& ovf, bool rg, const RangeS<NBOARD>& sin,
                                        const RangeS<NBOARD>& sout, float* rm_out,
                                        unsigned* ovw) {
    using G = GeoH<NBOARD, BS, 64 * CTW * H2_TM / F, ILV>;
    using C = CfgH<F, G::NPIX>;
    constexpr int KS = C::KS, CT = C::CT, NIT = C::NIT;
    // ILV: tile 0 is board row 0 (pixel group 0) or row 7 (group 1), and the taps with dr = -1
    // (row 0) or dr = +1 (row 7) leave the boards for all its pixels: tile 0's A loads and MFMAs
    // are skipped in those k-steps (1/12 of the conv MFMAs).
    // Both groups walk the taps in natural order, so the two waves of a channel group fetch the
    // same weight fragments at about the same time (L1 hits), and each skips in its own window,
    // group 0 in [0, 3 KS) (dr = -1), group 1 in [6 KS, 9 KS) (dr = +1), both compile-time: the
    // kernel instantiates the whole trunk once per group (GRP) behind one wave-uniform branch (190
    // VGPRs; the same choice made per layer needed 224, per k-step 248). Whole-bench A/B, one box:
    // +2.8% over a row-mirrored tap order in which both groups skip in the same window
    // (profiles/r02ah_ab_nat.txt; the mirrored orders lose the shared fragment fetches:
    // profiles/r02k_ab_h2_mirror_c2.json).
    const WaveTilesH<F, CTW, PTW> wt(wave, lane, ILV);
    // is tile 0 skipped in k-step i (compile-time once the k-loop is unrolled)
    auto skip0 = [](int i) -> bool {
        if (!ILV) return false;
        return GRP == 0 ? i < 3 * KS : (i >= 6 * KS && i < 9 * KS);
    };
    load_epi(er, bias, isc, wt, lane);                // lands during the k-loop
    const int kq = lane >> 4;                         // this lane's 8-channel slot in a k-step
    unsigned pmask[PTW];                              // valid taps in iteration order
#pragma unroll
    for (int u = 0; u < PTW; ++u) pmask[u] = G::taps(wt.px[u]);
    f32x4 acc[CTW][PTW];
#pragma unroll
    for (int c = 0; c < CTW; ++c)
#pragma unroll
        for (int u = 0; u < PTW; ++u) acc[c][u] = f32x4{};
    const int wu = wl + wt.ct0 * 64;
    auto load_b = [&](f16x8 (&bq)[CTW][2], int it) {
        const int f = wu + h2_frag<F>(it);
#pragma unroll
        for (int c = 0; c < CTW; ++c)
#pragma unroll
            for (int p = 0; p < 2; ++p) bq[c][p] = wr.load(f + (p * CT + c) * 64, lane);
    };
    auto load_a = [&](f16x8 (&aq)[PTW][2], int it) {
        const int t = it / KS, ks = it - t * KS;
        const int off = G::tap_offset(t);
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
    if constexpr (NIT <= 48) {   // F = 64, 128: the whole k-loop unrolled, one slot per k-step
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
            const int ia = it + APD;                  // the A operands loaded this k-step
            if (ia < NIT) load_a(aq[ia % (APD + 1)], ia);
            load_b(bq[it + PD], it + PD);
            const bool sa = ia < NIT && skip0(ia);    // next A load without tile 0
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
    } else {
        // F = 256 (72 k-steps of 48 MFMAs): a fully unrolled loop exceeds the unroller's budget
        // and a per-k-step register array indexed at run time lives in scratch. Weight fragments
        // rotate through PD + 1 slots and activations through APD + 1; the loop runs in chunks of
        // U k-steps (a multiple of both ring lengths), so every slot index inside a chunk is a
        // compile-time constant. No ILV here (one board per workgroup): no tile-0 skips.
        static_assert(!ILV, "the chunked k-loop has no tile-0 skip window");
        constexpr int RB = PD + 1, RA = APD + 1, U = 24;
        static_assert(NIT % U == 0 && U % RB == 0 && U % RA == 0, "k-loop chunking");
        f16x8 bq[RB][CTW][2];
        f16x8 aq[RA][PTW][2];
#pragma unroll
        for (int d = 0; d < PD; ++d)
#pragma unroll
            for (int c = 0; c < CTW; ++c)
#pragma unroll
                for (int p = 0; p < 2; ++p) bq[d][c][p] = bc[d][c][p];
#pragma unroll
        for (int d = 0; d < APD; ++d) load_a(aq[d], d);
#pragma unroll 1
        for (int o = 0; o < NIT; o += U) {
#pragma unroll
            for (int j = 0; j < U; ++j) {
                const int it = o + j, ia = it + APD;
                if (ia < NIT) load_a(aq[(j + APD) % RA], ia);
                load_b(bq[(j + PD) % RB], it + PD);
                mma3(acc, aq[j % RA], bq[j % RB]);
                interleave_loads<0, 3 * CTW * PTW, 2 * PTW, 2 * CTW>();
                __builtin_amdgcn_sched_barrier(0);
            }
        }
#pragma unroll
        for (int d = 0; d < PD; ++d)
#pragma unroll
            for (int c = 0; c < CTW; ++c)
#pragma unroll
                for (int p = 0; p < 2; ++p) bc[d][c][p] = bq[(NIT + d) % RB][c][p];
    }
    // conv A (block input -> t): the skip input stays in er.res; conv B adds it and keeps
    epilogue_h2<F, G::NPIX, CTW, PTW, RES, RES, G>(out, acc, er, wt, lane, wave, ovf, rg, sin, sout,
                                                   rm_out, ovw);
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
    // per board: the wave's max |input| -> rm[4 * b + wave] (RangeLds; the stem's bound)
    __device__ void maxima(float* rm, int tid, int wave) const {
#pragma unroll
        for (int b = 0; b < NBOARD; ++b) {
            float m = 0.0f;
#pragma unroll
            for (int j = 0; j < PER; ++j)
                m = (tid + j * NTHR) / 400 == b ? fmaxf(m, fabsf(v[j])) : m;
            m = wave_max_nonneg(m);
            if ((tid & 63) == 0) rm[4 * b + wave] = m;
        }
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

// The stem and the residual tower of one pass (h2_pass). RG (RANGED) false: every pass, values
// stored unscaled, boards that overflowed set their bit in the pass's overflow words; RG true: a
// re-run for those boards (mask) with the activation range scaled (RangeS), the others
// unscaled as before, so every row's outputs still depend only on its own position (the re-run
// prefetches one k-step of weights and no activations: its speed does not matter and its stack
// stays small). GR: the ILV pixel group (conv_h2's tile-0 skip window). Returns the final
// image's scale exponents.
template <int F, int NBOARD, int CTW, int PTW, int BS, bool ILV, int GR, bool RG>
__device__ __forceinline__ RangeS<NBOARD> h2_trunk(char* smem, const float* __restrict__ x,
                                                   const int (&gb)[NBOARD], const uint64_t* bits,
                                                   const float* __restrict__ prm, const Layout& L,
                                                   const uint16_t* __restrict__ blob,
                                                   int n_blocks, int tid, int lane, int wave,
                                                   bool& ovf, unsigned mask) {
    const BarWG bar{};
    using WT = WaveTilesH<F, CTW, PTW>;
    using G = GeoH<NBOARD, BS, 64 * CTW * H2_TM / F, ILV>;
    using C = CfgH<F, G::NPIX>;
    constexpr int NTHR = 256;
    uint16_t* actA = reinterpret_cast<uint16_t*>(smem);
    uint16_t* actB = actA + C::ACT;
    float* xin = reinterpret_cast<float*>(actB);     // free until the first conv writes B
    const H2W wr(blob, h2_blob_elems(F, n_blocks));
    const RangeLds rl{reinterpret_cast<float*>(smem + C::RMAX)};
    constexpr int PD = RG ? 1 : (F == 256 ? RVZ_H2_PD256 : RVZ_H2_PD), APD = RG ? 0 : RVZ_H2_APD;
    PASS_NOW(tp0);
    f16x8 bc[PD][CTW][2];
    if (n_blocks > 0) {
        const int wu = WT(wave, lane).ct0 * 64;
#pragma unroll
        for (int s = 0; s < PD; ++s) {
            const int f = wu + h2_frag<F>(s);
#pragma unroll
            for (int c = 0; c < CTW; ++c)
#pragma unroll
                for (int p = 0; p < 2; ++p) bc[s][c][p] = wr.load(f + (p * C::CT + c) * 64, lane);
        }
    }
    EpiH<CTW, PTW> er;
    f16x8 ws[CTW][2];
    // RANGED: {K, Bb} per layer from the blob's range table; the per-wave maxima in LDS
    // (RangeLds: slots 0 / 2 the inputs of even / odd blocks, 1 conv A's outputs); the
    // exponents of boards outside the mask forced to 0
    const float* rng = reinterpret_cast<const float*>(blob + h2_range_off(F, n_blocks));
    unsigned keep = 0;                            // 0xFF per masked board
#pragma unroll
    for (int k = 0; k < NBOARD; ++k) keep |= (mask >> k & 1u) ? 0xFFu << (8 * k) : 0u;
    auto masked = [&](RangeS<NBOARD> r) {
        r.pk &= (int)keep;
        return r;
    };
    auto bound = [&](const float (&m)[NBOARD], int l, const float* m_skip) {
        return RG ? masked(range_out(m, rng[2 * l], rng[2 * l + 1], m_skip)) : RangeS<NBOARD>{};
    };
    RangeS<NBOARD> simg;                          // the stored image's scale exponents
    float m_in[NBOARD];                           // (the stem's input maxima)
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
#pragma unroll
        for (int k = 0; k < NBOARD; ++k) m_in[k] = 1.0f;      // 0 / 1 planes
        simg = bound(m_in, 0, nullptr);
        stem_h2_bits<F, NBOARD, CTW, PTW, BS, ILV>(pl, actA, ws, wave, lane, er, ovf, RG, simg,
                                                       rl.slot(0), rl.ovw(wave));
    } else {
        XinStage<NBOARD, BS, NTHR> st;
        st.load(x, gb, tid);
        stem_h2_load<F, NBOARD, CTW, PTW>(blob, prm, L, n_blocks, wave, lane, er, ws);
        STEM_T(0);
        st.store(xin, tid);
        if constexpr (RG) st.maxima(rl.slot(1), tid, wave);
        STEM_T(1);
        bar();
        STEM_T(2);
        if constexpr (RG) {
#pragma unroll
            for (int k = 0; k < NBOARD; ++k) m_in[k] = rl.read(1, k);
            simg = bound(m_in, 0, nullptr);
        }
        stem_h2<F, NBOARD, CTW, PTW, BS, ILV>(xin, actA, ws, wave, lane, er, ovf, RG, simg,
                                                  rl.slot(0), rl.ovw(wave));
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
    for (int blk = 0; blk < n_blocks; ++blk) {
        const int l1 = 2 * blk, l2 = 2 * blk + 1, sb = 2 * (blk & 1);
        // conv A's output scale from the block input's maxima (slot sb; recomputed for conv B,
        // so nothing but the packed exponents lives across a conv)
        auto scale_t = [&] {
            float m[NBOARD];
#pragma unroll
            for (int k = 0; k < NBOARD; ++k) m[k] = RG ? rl.read(sb, k) : 0.0f;
            return bound(m, 1 + l1, nullptr);
        };
        conv_h2<F, NBOARD, CTW, PTW, false, BS, ILV, GR, PD, APD>(
            actA, actB, wr, (int)(l1 * LW / 8), prm + L.res_b + (size_t)l1 * F, isc + l1 * F,
            wave, lane, bc, er, ovf, RG, simg, scale_t(), rl.slot(1), rl.ovw(wave));
        if (blk == 0) PHASE(5);
        bar();
        if (blk == 0) PHASE(6);
        {
            float m_t[NBOARD], m_blk[NBOARD];
#pragma unroll
            for (int k = 0; k < NBOARD; ++k) {
                m_t[k] = RG ? rl.read(1, k) : 0.0f;
                m_blk[k] = RG ? rl.read(sb, k) : 0.0f;                // the skip input
            }
            const RangeS<NBOARD> st = scale_t();
            simg = bound(m_t, 1 + l2, m_blk);
            conv_h2<F, NBOARD, CTW, PTW, true, BS, ILV, GR, PD, APD>(
                actB, actA, wr, (int)(l2 * LW / 8), prm + L.res_b + (size_t)l2 * F,
                isc + l2 * F, wave, lane, bc, er, ovf, RG, st, simg, rl.slot(2 - sb),
                rl.ovw(wave));
        }
        bar();
    }
    return simg;
}

// The ranged re-run as a call: inlined next to the unscaled copy its registers pushed the hot
// path into spills; as a function the spills and the call's saves run only on the rare path.
template <int NBOARD>
struct BoardRows {                  // the pass's rows, by value (see h2_trunk_ranged)
    int v[NBOARD];
};
// Everything crosses the call by value (of the parameter layout only the two offsets the trunk
// reads) and the overflow flag comes back in the result: a reference argument (the Layout, the
// rows, the sticky flag) puts that object in scratch memory for the whole kernel, and the
// unscaled trunk then reads it from there (C1's one-board launches: -3.8%).
template <int F, int NBOARD, int CTW, int PTW, int BS, bool ILV, int GR>
__device__ __attribute__((noinline)) int2 h2_trunk_ranged(char* smem, const float* x,
                                                          BoardRows<NBOARD> rows,
                                                          const uint64_t* bits, const float* prm,
                                                          int64_t stem_b, int64_t res_b,
                                                          const uint16_t* blob, int n_blocks,
                                                          int tid, int lane, int wave,
                                                          unsigned mask) {
    Layout L{};                     // the trunk reads these two offsets of the parameter layout
    L.stem_b = stem_b;
    L.res_b = res_b;
    bool ovf = false;
    const RangeS<NBOARD> r = h2_trunk<F, NBOARD, CTW, PTW, BS, ILV, GR, true>(
        smem, x, rows.v, bits, prm, L, blob, n_blocks, tid, lane, wave, ovf, mask);
    return make_int2(r.pk, ovf ? 1 : 0);
}

// One pass of the workgroup (256 threads) over NBOARD boards: board b's leaf planes are row gb[b]
// of x ([rows][3][BS*BS], gb[b] < 0: no board), its 1x1 head-conv outputs go to row gb[b] of
// work ([rows][192]: policy planes, then the value plane). smem: CfgH<..>::BYTES of LDS, free on
// entry and on return. ovf |= an activation overflowed f16 (the caller's sticky word).
// Input of a pass: board b's leaf planes are row gb[b] of x (float [rows][3][BS*BS]), or, when
// bits is set, the bitboards bits[3 * b .. 3 * b + 2] = (P, O, V) (LDS). Output: the 1x1
// head-conv rows through hout (HeadsGlobalIdx: row gb[b] of work; HeadsInLds: the FC heads' LDS
// input rows).
template <int F, int NBOARD, int CTW, int PTW, int BS, class HOut>
__device__ __forceinline__ void h2_pass(char* smem, const float* __restrict__ x,
                                        const int (&gbv)[NBOARD], const uint64_t* bits,
                                        const float* __restrict__ prm, const Layout& L,
                                        const uint16_t* __restrict__ blob, int n_blocks,
                                        const HOut& hout, int tid, int lane, int wave, bool& ovf) {
    const BarWG bar{};
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
    // from the weight prefetch to the last residual block: ILV, one instance per pixel group
    // (its own tile-0 skip window, conv_h2), chosen by a wave-uniform branch
    const bool grp1 = ILV && wave / WT::CG != 0;
    const RangeLds rl{reinterpret_cast<float*>(smem + C::RMAX)};
    if (lane == 0) *rl.ovw(wave) = 0u;                // this wave's overflow word (its epilogues)
    // the stem and the residual tower. RANGED false: every pass, values stored unscaled, boards
    // that overflowed set their bit in the pass's overflow word; RANGED true: a re-run for those
    // boards (mask) with the activation range scaled (RangeS), the others unscaled as before,
    // so every row's outputs still depend only on its own position
    // (through a generic lambda: the same call written directly, or as a ?: pair, sends k_play's
    // packed 6x6 instance into 276 B of spills and C2's into 36 B — the inliner's order decides
    // which loop-invariant tap addresses stay hoisted; this form keeps round 4's codegen)
    auto trunk = [&](auto grp) -> RangeS<NBOARD> {
        constexpr int GR = decltype(grp)::value;
        return h2_trunk<F, NBOARD, CTW, PTW, BS, ILV, GR, false>(smem, x, gb, bits, prm, L, blob,
                                                                 n_blocks, tid, lane, wave, ovf, 0u);
    };
    RangeS<NBOARD> simg;
    if (grp1)
        simg = trunk(std::integral_constant<int, 1>{});
    else
        simg = trunk(std::integral_constant<int, 0>{});
    // the overflow words are final after the tower's last barrier (n_blocks = 0: the stem's)
    const unsigned omask = rl.ov_all();
    if (omask != 0u) {                                // rare: re-run the boards that overflowed
        __syncthreads();                              // every wave has read the words
        BoardRows<NBOARD> rows;
#pragma unroll
        for (int k = 0; k < NBOARD; ++k) rows.v[k] = gb[k];
        const int2 r =
            grp1 ? h2_trunk_ranged<F, NBOARD, CTW, PTW, BS, ILV, 1>(
                       smem, x, rows, bits, prm, L.stem_b, L.res_b, blob, n_blocks, tid, lane,
                       wave, omask)
                 : h2_trunk_ranged<F, NBOARD, CTW, PTW, BS, ILV, 0>(
                       smem, x, rows, bits, prm, L.stem_b, L.res_b, blob, n_blocks, tid, lane,
                       wave, omask);
        simg.pk = r.x;
        ovf |= r.y != 0;
    }
    PHASE(2);
    PASS_NOW(tp2);
    PASS_ADD(1, tp2 - tp0);   // stem + tower
    // the 1x1 head convs -> work (the FC heads are the next launch, k_heads_mfma)
    const ActH2<F, G::NPIX> act{actA, simg.pk};
    head_convs<F, NBOARD, NTHR, BS, true, ILV>(act, reinterpret_cast<float*>(actB), prm, L, hout,
                                              tid, bar);
#ifdef RVZ_PLAY_TIMING
    {
        PASS_NOW(tp3);
        PASS_ADD(2, tp3 - tp2);
        PASS_ADD(3, 1);
    }
#endif
}

// bits 52-55 of a workgroup's end stamp: the XCD it ran on (HW_REG_XCC_ID; bench.py --stamps-dump)
__device__ __forceinline__ uint64_t stamp_xcc() {
    return (uint64_t)(__builtin_amdgcn_s_getreg((31 << 11) | 20) & 0xF) << 52;
}
}  // namespace
