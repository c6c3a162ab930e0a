// rvz_resnet.hip — the reference's policy/value ResNet forward (network.py:30-117, BN folded) as
// the rvz leaf evaluator on gfx950: ONE trunk kernel per leaf batch (k_resnet_h2: stem, residual
// tower and 1x1 head convs, activations resident in LDS) plus one batched FC-heads launch
// (k_heads_mfma, rvz_resnet_common.hip.h), fp32-class arithmetic on the f16 matrix cores.
//
// Why one kernel: with MIOpen, every conv layer is a separate launch plus a zero-fill of its
// output and a bias/skip/ReLU pass, and every activation makes an HBM round trip. Here a
// workgroup keeps its boards' activations in LDS for the whole network: HBM traffic is the leaf
// planes in and the head-conv outputs out; weights stream from L2 (shared by every workgroup).
// The A/B alternatives (exact f32 MFMA, 3-part bf16 split, VALU heads, the MIOpen epilogue) are
// built into tools/alt/librvz_alt.so, not into this library.
#include "rvz_h2.hip.h"
#include "rvz_trace.h"

namespace {

template <int F, int NBOARD, int CTW, int PTW, int BS, int OCC>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC, OCC)))
void k_resnet_h2(const float* __restrict__ x, int n_boards, const float* __restrict__ prm,
                 Layout L, const uint16_t* __restrict__ blob, int n_blocks,
                 float* __restrict__ work, const int32_t* __restrict__ n_live,
                 uint64_t* __restrict__ stamps, const uint32_t* __restrict__ stamp_ctr,
                 int ring, unsigned long long* __restrict__ claim) {
    using WT = WaveTilesH<F, CTW, PTW>;
    // row-interleaved pair of 8x8 boards (GeoH ILV): two pixel groups of 4 tiles = 8 board rows
    constexpr bool ILV = RVZ_H2_ILV && NBOARD == 2 && BS == 8 && PTW == 4 && WT::CG == 2;
    using G = GeoH<NBOARD, BS, 64 * CTW * H2_TM / F, ILV>;
    using C = CfgH<F, G::NPIX>;
    static_assert(WT::CG * (G::NPIX / (PTW * H2_TN)) == 4, "4 waves");
    static_assert(1024 * 4 <= C::ACT * 2, "head-conv partial sums fit in B");
    static_assert(NBOARD * 100 * 4 * 4 <= C::ACT * 2, "xin fits in buffer B");
    __shared__ __attribute__((aligned(16))) char smem[C::BYTES];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    int unit = blockIdx.x;
    if (claim) {
        // RVZ_H2_DYN: board units are dealt in workgroup start order from a counter in the
        // workspace, over a grid larger than the units; the workgroups that start last (on the
        // XCDs that run slowest) find none left and exit. The 64-bit counter is never reset: each
        // launch adds exactly gridDim.x, so claim mod gridDim.x covers every unit once per launch
        // whatever the counter held below 2^63 (a zeroed workspace keeps the spare units last).
        __shared__ int s_unit;
        if (tid == 0) {
            s_unit = (int)(atomicAdd(claim, 1ull) % gridDim.x);
        }
        __syncthreads();
        unit = s_unit;
    }
    const int g0 = unit * NBOARD;
    bool ovf = false;
    // optional device timestamps (bench.py: the launch's span inside a replayed HIP graph):
    // s_memrealtime (100 MHz) at the workgroup's start and end
    // row of a ring of launches when stamp_ctr is given (advanced by the heads launch)
    uint64_t t_start = 0;
    if (stamps) {
        t_start = __builtin_amdgcn_s_memrealtime();
        const uint32_t slot = stamp_ctr ? *stamp_ctr % (uint32_t)ring : 0u;
        stamps += ((size_t)slot * gridDim.x + blockIdx.x) * 2;
    }
    // a compacted leaf batch (rvz_search_compact): dead boards are not evaluated, their rows are
    // never read (a unit of dead boards exits before the first barrier; a unit across a stripe
    // end (NBOARD not dividing the stripe) evaluates its live boards only)
    int gb[NBOARD];
    int n_eval = 0;
#pragma unroll
    for (int k = 0; k < NBOARD; ++k) {
        const bool live = g0 + k < n_boards && !row_dead(n_live, g0 + k);
        gb[k] = live ? g0 + k : -1;
        n_eval += live ? 1 : 0;
    }
    if (n_eval == 0) {
        if (stamps && tid == 0) {
            stamps[0] = t_start;
            stamps[1] = __builtin_amdgcn_s_memrealtime() | stamp_xcc();
        }
        return;
    }
    PHASE(0);
    RT(0);
    HWID();
    h2_pass<F, NBOARD, CTW, PTW, BS>(smem, x, gb, nullptr, prm, L, blob, n_blocks,
                                     HeadsGlobalIdx<NBOARD>(work, gb), tid, lane, wave, ovf);
    PHASE(3);
    RT(1);
    if (ovf) work[(size_t)n_boards * 192] = 1.0f;   // benign race: every writer stores 1
    if (stamps) {   // end stamp; bits 56-63: the workgroup's live boards (bench.py's FLOPs)
        const uint64_t nb = (uint64_t)n_eval;
        __syncthreads();
        if (tid == 0) {
            stamps[0] = t_start;
            stamps[1] = __builtin_amdgcn_s_memrealtime() | stamp_xcc() | (nb << 56);
        }
    }
}

// per (layer, out-channel) wave: scale = 2^(14 - floor(log2 max|w|)), split the scaled weights
// into the fragment layout, store 1/scale. Layer -1 (blockIdx.y == 0) is the stem.
// The stem's K order (k_resnet_h2 stem_h2): slot k of lane group g = k / 8 holds tap 2g channels
// 0-2 (s = k % 8 < 3), tap 2g + 1 channels 0-2 (s < 6); the ninth tap fills the spare slots:
// group 0 s = 6, 7 -> tap 8 channels 0, 1; group 1 s = 6 -> tap 8 channel 2. Returns tap * 3 +
// channel, or -1 for a zero slot. A lane then reads whole (tap) float4s of the padded input.
__host__ __device__ constexpr int h2_stem_slot(int k) {
    const int g = k / 8, s = k % 8;
    return s < 3   ? (2 * g) * 3 + s
           : s < 6 ? (2 * g + 1) * 3 + (s - 3)
           : (g == 0 ? 24 + (s - 6) : (g == 1 && s == 6 ? 26 : -1));
}

__global__ __launch_bounds__(64) void k_h2_weights(const float* __restrict__ prm, Layout L, int F,
                                                   int NB, uint16_t* __restrict__ blob) {
    const int n = blockIdx.x, lyr = (int)blockIdx.y - 1, lane = threadIdx.x;
    const int CT = F / H2_TM, KS = F / H2_K;
    const int cnt = lyr < 0 ? 27 : 9 * F;
    auto wget = [&](int i) -> float {   // i = tap*F + k (trunk) or k (stem)
        if (lyr < 0) return prm[L.stem_w + (int64_t)n * 27 + i];
        const int t = i / F, k = i % F;
        return prm[L.res_w + (((int64_t)lyr * 9 + t) * F + n) * F + k];
    };
    float m = 0.0f, l1 = 0.0f;
    for (int i = lane; i < cnt; i += 64) {
        m = fmaxf(m, fabsf(wget(i)));
        l1 += fabsf(wget(i));
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        m = fmaxf(m, __shfl_xor(m, o));
        l1 += __shfl_xor(l1, o);
    }
    if (lane == 0) {   // the activation-range table: max over channels (non-negative floats
                       // order as their bit patterns: an unsigned max, zeroed by the host first)
        unsigned* rng = reinterpret_cast<unsigned*>(blob + h2_range_off(F, NB)) + 2 * (lyr + 1);
        const float b = lyr < 0 ? prm[L.stem_b + n] : prm[L.res_b + (int64_t)lyr * F + n];
        atomicMax(rng, __float_as_uint(l1));
        atomicMax(rng + 1, __float_as_uint(fabsf(b)));
    }
    int e = 0;
    if (m > 0.0f) {
        frexpf(m, &e);                         // m = f * 2^e, f in [0.5, 1): floor(log2 m) = e - 1
        e = 14 - (e - 1);
        e = e < -100 ? -100 : (e > 100 ? 100 : e);
    }
    const float sc = ldexpf(1.0f, e);
    float* isc = reinterpret_cast<float*>(blob + h2_scale_off(F, NB));
    if (lane == 0) isc[(lyr + 1) * F + n] = ldexpf(1.0f, -e);
    const int ct = n / H2_TM;
    if (lyr < 0) {                             // stem: [part][ct][lane][8], k < 32
        uint16_t* o = blob + h2_stem_off(F, NB);
        if (lane < 32) {
            const int k = lane, ln = (k / 8) * H2_TM + n % H2_TM, ix = h2_stem_slot(k);
            const float w = ix >= 0 ? wget(ix) * sc : 0.0f;
            const _Float16 h0 = (_Float16)w;
            const _Float16 h1 = (_Float16)(w - (float)h0);
            o[((0 * CT + ct) * 64 + ln) * 8 + k % 8] = __builtin_bit_cast(uint16_t, h0);
            o[((1 * CT + ct) * 64 + ln) * 8 + k % 8] = __builtin_bit_cast(uint16_t, h1);
        }
        return;
    }
    for (int i = lane; i < cnt; i += 64) {
        const int t = i / F, k = i % F, ks = k / H2_K, ln = ((k % H2_K) / 8) * H2_TM + n % H2_TM;
        const float w = wget(i) * sc;
        const _Float16 h0 = (_Float16)w;
        const _Float16 h1 = (_Float16)(w - (float)h0);
        const int64_t base = (((int64_t)lyr * 9 + t) * KS + ks) * 2;
        blob[(((base + 0) * CT + ct) * 64 + ln) * 8 + k % 8] = __builtin_bit_cast(uint16_t, h0);
        blob[(((base + 1) * CT + ct) * 64 + ln) * 8 + k % 8] = __builtin_bit_cast(uint16_t, h1);
    }
}
}  // namespace

// workgroups of one h2 trunk launch (k_resnet_h2's grid)
// RVZ_H2_DYN 1 (default): board units dealt to workgroups in start order (k_resnet_h2, `claim`).
// Under this load the eight XCDs hold different clocks (1.73-1.92 GHz, power-limited at ~1.3 kW;
// profiles/r02ac_power.txt), and blocks are dealt round-robin over the XCDs, so with one unit per
// block the slowest XCD set the pace and the faster ones idled at the end of every launch. With
// 1/8 spare workgroups the faster XCDs take more units: C2 +2.2%, C3 +2.5%, C5 +2.2%
// (whole-bench A/Bs, profiles/r02ad_ab_dyn.txt).
#ifndef RVZ_H2_DYN
#define RVZ_H2_DYN 1
#endif
#ifndef RVZ_H2_C5NB
#define RVZ_H2_C5NB 3         // packed 6x6 at F = 64: boards per workgroup (3: 108 of 128 rows, two
#endif                        // workgroups per CU, the 8x8 pair's tile map; 4: 160 rows, 1 per CU,
                              // C5 -0.7%; 2: 96 rows, -12%)
#ifndef RVZ_H2_SPARE
#define RVZ_H2_SPARE 8        // 1/RVZ_H2_SPARE spare workgroups (a multiple of 8, at least 8)
#endif
// board units of one h2 trunk launch, and its grid (RVZ_H2_DYN: + 1/RVZ_H2_SPARE spare workgroups)
static int h2_units(int bs, int filters, int n) {
    if (bs == 6) return filters == 64 ? (n + RVZ_H2_C5NB - 1) / RVZ_H2_C5NB : n;
    return filters == 64 ? (n + 1) / 2 : n;
}
static int h2_grid(int bs, int filters, int n) {
    const int u = h2_units(bs, filters, n);
    return RVZ_H2_DYN && u > 0 ? u + ((u + 8 * RVZ_H2_SPARE - 1) / (8 * RVZ_H2_SPARE)) * 8 : u;
}

template <int BS>
static void launch_trunk_h2(const float* x, int32_t n, const float* params, const uint16_t* blob,
                            int32_t filters, int32_t blocks, float* work, hipStream_t s,
                            const int32_t* n_live, uint64_t* stamps, const uint32_t* stamp_ctr,
                            int ring) {
    const Layout L = make_layout(filters, blocks, BS);
    const dim3 grid(h2_grid(BS, filters, n));
    // the unit counter: words n*192 + 2, 3 of the workspace (8-byte aligned)
    unsigned long long* claim =
        RVZ_H2_DYN ? reinterpret_cast<unsigned long long*>(work + (size_t)n * 192 + 2) : nullptr;
    if (BS == 6) {   // packed 6x6: F=64 3 boards = 128 pixel rows (8 tiles); F=128 1 board = 48
        if (filters == 64)
            hipLaunchKernelGGL((k_resnet_h2<64, RVZ_H2_C5NB, 2, (RVZ_H2_C5NB * 36 + 31) / 32,
                                            6, RVZ_H2_C5NB == 4 ? 1 : 2>), grid, dim3(256), 0, s, x, n,
                               params, L, blob, blocks, work, n_live, stamps, stamp_ctr, ring,
                               claim);
        else
            hipLaunchKernelGGL((k_resnet_h2<128, 1, 2, 3, 6, 2>), grid, dim3(256), 0, s, x, n,
                               params, L, blob, blocks, work, n_live, stamps, stamp_ctr, ring,
                               claim);
    } else if (filters == 64)
        hipLaunchKernelGGL((k_resnet_h2<64, 2, 2, 4, 8, 2>), grid, dim3(256), 0, s, x, n,
                           params, L, blob, blocks, work, n_live, stamps, stamp_ctr, ring,
                           claim);
    else if (filters == 128)
        hipLaunchKernelGGL((k_resnet_h2<128, 1, 2, 4, 8, 2>), grid, dim3(256), 0, s, x, n, params,
                           L, blob, blocks, work, n_live, stamps, stamp_ctr, ring, claim);
    else   // F=256: the F=128 tile map with 4 channel tiles per wave; 144 KB of LDS, 1 per CU
        hipLaunchKernelGGL((k_resnet_h2<256, 1, 4, 4, 8, 1>), grid, dim3(256), 0, s, x, n, params,
                           L, blob, blocks, work, n_live, stamps, stamp_ctr, ring, claim);
}

extern "C" {

static bool board_ok(int32_t bs) { return bs == 8 || bs == 6; }
// trunk widths with an h2 instantiation: 64 and 128 on both boards, 256 on 8x8
static bool width_ok(int32_t filters) { return filters == 64 || filters == 128 || filters == 256; }
static bool trunk_ok(int32_t bs, int32_t filters) {
    return board_ok(bs) && (filters == 64 || filters == 128 || (filters == 256 && bs == 8));
}

int64_t rvz_resnet_params_size(int32_t board, int32_t filters, int32_t blocks) {
    if (!width_ok(filters) || blocks < 0 || !board_ok(board)) return RVZ_EINVAL;
    return make_layout(filters, blocks, board).total;
}
#ifdef RVZ_PHASE_TIMING
int rvz_hwid_read(uint32_t* host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_hwid), (size_t)n * 2 * sizeof(uint32_t)) ==
                   hipSuccess ? 0 : -5;
}
int rvz_stem_read(uint64_t* host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stem), (size_t)n * 8 * sizeof(uint64_t)) ==
                   hipSuccess ? 0 : -5;
}
int rvz_rt_read(uint64_t* host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_rt), (size_t)n * 2 * sizeof(uint64_t)) ==
                   hipSuccess ? 0 : -5;
}
int rvz_wave_read(uint64_t* host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_wave), (size_t)n * 16 * sizeof(uint64_t)) ==
                   hipSuccess ? 0 : -5;
}
int rvz_phase_read(uint64_t* host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_phase), (size_t)n * 8 * sizeof(uint64_t)) ==
                   hipSuccess ? 0 : -5;
}
#endif
// + 4 floats: word n*192 is the h2 kernel's sticky activation-overflow flag (zero it before the
// first launch), words n*192 + 2, 3 its 64-bit unit counter (RVZ_H2_DYN; any value below 2^63)
int64_t rvz_resnet_work_size(int32_t n) { return n < 0 ? RVZ_EINVAL : (int64_t)n * 192 + 4; }
int rvz_resnet_heads_fc_ex(int32_t board, const float* work, int32_t n, const float* params,
                           int32_t filters, int32_t blocks, float* logits, float* value,
                           const int32_t* n_live, uint32_t* stamp_ctr, void* stream) {
    const rvz::Range trace_range("rvz.eval.heads (k_heads_mfma)");
    if (!work || !params || !logits || !value || n < 0 || blocks < 0 || !board_ok(board) ||
        !width_ok(filters))
        return RVZ_EINVAL;
    // the heads copy workspace rows as f32x4: a misaligned workspace is an argument error, not
    // a device fault
    if (((uintptr_t)params & 15) != 0 || ((uintptr_t)work & 15) != 0) return RVZ_EINVAL;
    if (n == 0) return RVZ_OK;
    const Layout L = make_layout(filters, blocks, board);
    const dim3 grid((n + 15) / 16), block(256);
    if (board == 8)
        hipLaunchKernelGGL(k_heads_mfma<8>, grid, block, 0, (hipStream_t)stream, work, n, params,
                           L, logits, value, n_live, stamp_ctr);
    else
        hipLaunchKernelGGL(k_heads_mfma<6>, grid, block, 0, (hipStream_t)stream, work, n, params,
                           L, logits, value, n_live, stamp_ctr);
    return hipGetLastError() == hipSuccess ? RVZ_OK : RVZ_EHIP;
}

int rvz_resnet_heads_fc(int32_t board, const float* work, int32_t n, const float* params,
                        int32_t filters, int32_t blocks, float* logits, float* value,
                        void* stream) {
    return rvz_resnet_heads_fc_ex(board, work, n, params, filters, blocks, logits, value, nullptr,
                                  nullptr, stream);
}
int64_t rvz_resnet_h2_size(int32_t filters, int32_t blocks) {
    if (!width_ok(filters) || blocks < 0) return RVZ_EINVAL;
    return h2_blob_elems(filters, blocks);
}

int rvz_resnet_h2_weights(const float* params, int32_t filters, int32_t blocks, uint16_t* blob,
                          void* stream) {
    if (!params || !blob || !width_ok(filters) || blocks < 0) return RVZ_EINVAL;
    if (((uintptr_t)blob & 15) != 0) return RVZ_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    const Layout L = make_layout(filters, blocks);
    // the prefetch padding after the last layer reads zeros
    if (hipMemsetAsync(blob + 2 * blocks * h2_layer_elems(filters), 0,
                       h2_pad_ksteps(filters) * h2_kstep_elems(filters) * 2, s) != hipSuccess)
        return RVZ_EHIP;
    // the activation-range table is a max over the launch's workgroups: zeroed first
    if (hipMemsetAsync(blob + h2_range_off(filters, blocks), 0,
                       (h2_blob_elems(filters, blocks) - h2_range_off(filters, blocks)) * 2,
                       s) != hipSuccess)
        return RVZ_EHIP;
    hipLaunchKernelGGL(k_h2_weights, dim3(filters, 1 + 2 * blocks), dim3(64), 0, s, params, L,
                       (int)filters, (int)blocks, blob);
    return hipGetLastError() == hipSuccess ? RVZ_OK : RVZ_EHIP;
}

int rvz_resnet_trunk_h2_ex(int32_t board, const float* x, int32_t n, const float* params,
                           const uint16_t* blob, int32_t filters, int32_t blocks, float* work,
                           const int32_t* n_live, uint64_t* stamps, const uint32_t* stamp_ctr,
                           int32_t ring, void* stream) {
    const rvz::Range trace_range("rvz.eval.trunk (k_resnet_h2)");
    if (!x || !params || !blob || !work || n < 0 || blocks < 0 || !trunk_ok(board, filters) ||
        (stamp_ctr && (!stamps || ring <= 0)))
        return RVZ_EINVAL;
    // work: 16-byte aligned (the 64-bit unit-counter atomic at words n*192 + 2, 3 and the
    // heads' f32x4 row copies)
    if (((uintptr_t)params & 15) != 0 || ((uintptr_t)blob & 15) != 0 ||
        ((uintptr_t)work & 15) != 0)
        return RVZ_EINVAL;
    if (n == 0) return RVZ_OK;
    hipStream_t s = (hipStream_t)stream;
    if (board == 8)
        launch_trunk_h2<8>(x, n, params, blob, filters, blocks, work, s, n_live,
                           stamps, stamp_ctr, ring > 0 ? ring : 1);
    else
        launch_trunk_h2<6>(x, n, params, blob, filters, blocks, work, s, n_live,
                           stamps, stamp_ctr, ring > 0 ? ring : 1);
    return hipGetLastError() == hipSuccess ? RVZ_OK : RVZ_EHIP;
}

int rvz_resnet_trunk_h2(int32_t board, const float* x, int32_t n, const float* params,
                        const uint16_t* blob, int32_t filters, int32_t blocks, float* work,
                        void* stream) {
    return rvz_resnet_trunk_h2_ex(board, x, n, params, blob, filters, blocks, work, nullptr,
                                  nullptr, nullptr, 0, stream);
}

int32_t rvz_resnet_h2_grid(int32_t board, int32_t filters, int32_t n) {
    if (!trunk_ok(board, filters) || n < 0) return RVZ_EINVAL;
    return h2_grid(board, filters, n);
}

int rvz_resnet_fwd_h2_ex(int32_t board, const float* x, int32_t n, const float* params,
                         const uint16_t* blob, int32_t filters, int32_t blocks, float* work,
                         float* logits, float* value, const int32_t* n_live, void* stream) {
    if (!logits || !value) return RVZ_EINVAL;
    const int rc = rvz_resnet_trunk_h2_ex(board, x, n, params, blob, filters, blocks, work, n_live,
                                          nullptr, nullptr, 0, stream);
    if (rc != RVZ_OK) return rc;
    return rvz_resnet_heads_fc_ex(board, work, n, params, filters, blocks, logits, value, n_live,
                                  nullptr, stream);
}

int rvz_resnet_fwd_h2(int32_t board, const float* x, int32_t n, const float* params,
                      const uint16_t* blob, int32_t filters, int32_t blocks, float* work,
                      float* logits, float* value, void* stream) {
    return rvz_resnet_fwd_h2_ex(board, x, n, params, blob, filters, blocks, work, logits, value,
                                nullptr, stream);
}

}  // extern "C"