// rvz_engine.hip — batched Reversi env + lockstep reference-semantics PUCT for gfx950 (MI355X),
// exported through the C-ABI in include/rvz.h.
//
// Layout (HBM, per engine of G games):
//   env    black[G], white[G] (u64), status[G][4] (side, over, winner, passed)
//   tree   nodes[G][M] {N i32, W f32, P f32, C f32}, meta[G][M] u32, M = 1 + E*S*S,
//          E = ceil(sims / batch) = expansions per search; node 0 = root, expansion e of a search
//          owns the child block [1 + e*S*S, 1 + (e+1)*S*S), children in row-major square order.
//   search path[G][64] i32, pend[G] (queued copies), plen[G], leaf_legal[G] u64, nexp[G]
//   rng    u[G][64] f64: np.random.random_sample() stream of each game's seed, pos[G]
//
// One wavefront per game in every search kernel: lane i owns child i (UCB, expansion) or
// square i (planes, visits, policy), so a 64-square board is exactly one wave.
//
// Exactness notes (mirrored and checked by oracle/rvz_oracle.c, which keeps the literal rules):
//  * Within a batch every traversal of a game follows the same path (UCB scores are cached and only
//    invalidated by a backup of that node, mcts.py:99-113,639-640; unvisited children score +inf,
//    mcts.py:96-97), unless a traversal ends on an already-known terminal, which is backed up at
//    once (mcts.py:364-366). select therefore walks once per terminal hit plus once for the
//    queued leaf, and backs the NN value up `copies` times (B sequential fp32 adds).
//  * Virtual loss is always 0 when a score is computed (every traversal that scores starts from a
//    balanced tree), so u = c*P*sqrt(Np) / (1 + N).
//  * value_sum is float32 (NumPy>=2 promotion of the np.float32 NN value); terminal values are
//    small integers, exact in float32, so one float32 accumulator reproduces the Python mix.
//  * sqrt(Np) is the correctly rounded f32 sqrt of (float)n (sqrt_count): equal to math.sqrt in
//    double then the float32 cast (double rounding through >= 2p + 2 bits is innocuous for
//    sqrt; tests/test_gpu_numerics.py checks every n <= 4,000,000), at f32 cost.
#include <hip/hip_bf16.h>
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/rvz.h"
#include "rvz_h2.hip.h"
#include "rvz_pow.hip.h"
#include "rvz_rules.hip.h"
#include "rvz_trace.h"

using namespace rvz;

namespace {

constexpr int WAVE = 64;
constexpr int WPB = 4;            // waves (games) per 256-thread workgroup
constexpr int PATH_CAP = 64;      // path length limit: ceil(sims / batch) <= 64
constexpr int RNG_DRAWS = 64;     // random_sample() values per seed (a game has <= 60 plies)

struct Node {
    int32_t n;   // visit_count
    float w;     // value_sum
    float p;     // prior
    float c;     // cached_ucb; NaN = not cached
};
static_assert(sizeof(Node) == 16, "node is one 16-byte load");

// meta word: sq[0:6) turn[6:8) terminal[8] tv[9:11) (0: 0.0, 1: +1.0, 2: -1.0) nchild[11:18) block[18:32)
__host__ __device__ constexpr uint32_t meta_pack(int sq, int turn) {
    return (uint32_t)(sq & 63) | ((uint32_t)(turn & 3) << 6);
}
__device__ __forceinline__ int m_sq(uint32_t m) { return (int)(m & 63u); }
__device__ __forceinline__ int m_turn(uint32_t m) { return (int)((m >> 6) & 3u); }
__device__ __forceinline__ bool m_term(uint32_t m) { return (m >> 8) & 1u; }
__device__ __forceinline__ float m_tv(uint32_t m) {
    const uint32_t t = (m >> 9) & 3u;
    return t == 1u ? 1.0f : (t == 2u ? -1.0f : 0.0f);
}
__device__ __forceinline__ int m_nchild(uint32_t m) { return (int)((m >> 11) & 127u); }
__device__ __forceinline__ int m_block(uint32_t m) { return (int)(m >> 18); }

struct View {  // kernel argument: device pointers + sizes
    int G, M;
    float cpuct;
    uint64_t* black;
    uint64_t* white;
    int32_t* status;  // [G][4]
    Node* nodes;
    uint32_t* meta;
    int32_t* path;  // [G][PATH_CAP]
    int32_t* pend;
    int32_t* plen;
    uint64_t* leaf_legal;
    uint64_t* root_legal;  // [G] legal mask of the current search's root (its children's squares)
    uint32_t* leaf_meta;   // [G] meta word of the queued leaf (written by select, read by expand)
    int32_t* nexp;
    double* rng_u;          // [G][RNG_DRAWS]
    int32_t* rng_pos;
    int32_t* err;
    unsigned long long* stats;  // [3][G] algorithmic bytes per game: k_step, k_act, k_expand_backup; or null
    // compacted leaf batches (rvz_search_compact), or null: live[(e * NS + s) * PITCH] = live
    // leaves of stripe s (games [s*STRIPE, (s+1)*STRIPE)) in batch e of the current search, at
    // rows [s*STRIPE, s*STRIPE + count) of leaf_x; row_of[g] = game g's row
    int32_t* live;   // [E][NS][PITCH]
    int32_t* row_of;  // [G]
    unsigned long long* live_total;  // running sum of the live counts (rows handed out)
    int E, NS;
    // NN-output memo across consecutive searches (rvz_search_memo; memo = 0: off). The pool has
    // two halves of E expansion blocks; a search writes one half while the previous search's
    // tree stays readable in the other. bval[g][b]: the NN value of the node expanded into block
    // b; carry[g]: the link (LINK_* below) of the child the last move went to, or LINK_NONE.
    int memo;
    uint32_t* carry;  // [G]
    float* bval;      // [G][2E]
};

// A link names an expanded node of the previous search's tree (the same position as the new
// node it is attached to): its index, child count and block. Stored in the `c` (cached UCB) field
// of an unvisited node, which the reference formula never reads while N == 0 (mcts.py:96-97;
// the first backup overwrites it with "not cached"), and in carry[g] for the next root.
// LINK_NONE is the "not cached" NaN every other node carries; a link is < 2^28, never a NaN.
constexpr uint32_t LINK_NONE = 0x7fc00000u;
__host__ __device__ constexpr uint32_t link_pack(int node, int nchild, int block) {
    return (uint32_t)node | ((uint32_t)nchild << 14) | ((uint32_t)block << 21);
}
__device__ __forceinline__ bool link_ok(uint32_t l) { return l < (1u << 28); }
__device__ __forceinline__ int link_node(uint32_t l) { return (int)(l & 0x3fffu); }
__device__ __forceinline__ int link_nchild(uint32_t l) { return (int)((l >> 14) & 127u); }
__device__ __forceinline__ int link_block(uint32_t l) { return (int)((l >> 21) & 127u); }

// ERR_NN: an evaluator handed the expand a non-finite value or probability (an overflowed or
// broken leaf evaluator must not feed the tree silently; the reference would play on with NaN)
enum : int32_t { ERR_RNG = 1, ERR_POOL = 2, ERR_PATH = 4, ERR_NN = 8 };

// Walk counters of the select phase per game (instrumented builds only, -DRVZ_WALK_STATS:
// tools/exp_walks.py): [0] walks from the root, [1] tree levels read, [2] known-terminal hits
// backed up in memory, [3] hits taken by the register fast path, [4] new terminals found
#ifdef RVZ_WALK_STATS
constexpr int WALK_STATS_MAX = 1 << 16;
__device__ unsigned int g_walk[WALK_STATS_MAX][5];
#define WALK_STAT(i, k) \
    if (lane == 0 && g < WALK_STATS_MAX) g_walk[g][i] += (k)
// shader-clock split of a game's k_step work: [0] expand phase (k_play: the cross-game table
// lookups), [1] walk levels, [2] memory backups of known terminals, [3] register fast path,
// [4] leaf (position, legal moves, queue)
__device__ unsigned long long g_wtime[WALK_STATS_MAX][5];
#define WT_NOW(t) const uint64_t t = __builtin_amdgcn_s_memtime()
#define WT_ADD(i, t0) \
    if (lane == 0 && g < WALK_STATS_MAX) g_wtime[g][i] += __builtin_amdgcn_s_memtime() - (t0)
// the fused kernel's game steps (k_play, tools/exp_play_walks.py): [0] expand, [1] act +
// autoreset, [2] the whole step (a game's turn in one search phase), [3] steps
__device__ unsigned long long g_ftime[WALK_STATS_MAX][4];
#define FT_ADD(i, t0) \
    if (lane == 0 && g < WALK_STATS_MAX) g_ftime[g][i] += __builtin_amdgcn_s_memtime() - (t0)
#define FT_CNT() \
    if (lane == 0 && g < WALK_STATS_MAX) g_ftime[g][3] += 1
#else
#define FT_ADD(i, t0)
#define FT_CNT()
#define WALK_STAT(i, k)
#define WT_NOW(t)
#define WT_ADD(i, t0)
#endif

__device__ __forceinline__ GameS load_game(const View& v, int g) {
    GameS s;
    s.black = v.black[g];
    s.white = v.white[g];
    const int4 st = reinterpret_cast<const int4*>(v.status)[g];
    s.side = st.x; s.over = st.y; s.winner = st.z; s.passed = st.w;
    return s;
}
__device__ __forceinline__ void store_game(const View& v, int g, const GameS& s) {
    v.black[g] = s.black;
    v.white[g] = s.white;
    reinterpret_cast<int4*>(v.status)[g] = make_int4(s.side, s.over, s.winner, s.passed);
}

// ---- wave primitives --------------------------------------------------------------------------
__device__ __forceinline__ int wave_sum_i(int x) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o);
    return x;
}
__device__ __forceinline__ float wave_sum_f(float x) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o);
    return x;
}
// Order key of a non-NaN score for an unsigned max (-0.0 ties +0.0).
__device__ __forceinline__ uint32_t score_key(float s) {
    const uint32_t b = __float_as_uint(s == 0.0f ? 0.0f : s);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
// Unsigned max over the wave on the DPP network (row shifts, then row broadcasts; lane 63 ends
// with the total): no LDS crossbar traffic, unlike __shfl_xor (ds_bpermute).
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t x) {
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false));  // row_shr:1
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false));  // row_shr:2
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false));  // row_shr:4
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false));  // row_shr:8
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false));  // row_bcast:15
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false));  // row_bcast:31
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}
// fmaxf over the wave on the DPP network (order-independent: max is exact)
__device__ __forceinline__ float wave_max_f(float x) {
    const int ninf = (int)0xff800000u;   // -inf: the identity of the lanes a shift leaves empty
    x = fmaxf(x, __int_as_float(__builtin_amdgcn_update_dpp(ninf, __float_as_int(x), 0x111, 0xf, 0xf, false)));
    x = fmaxf(x, __int_as_float(__builtin_amdgcn_update_dpp(ninf, __float_as_int(x), 0x112, 0xf, 0xf, false)));
    x = fmaxf(x, __int_as_float(__builtin_amdgcn_update_dpp(ninf, __float_as_int(x), 0x114, 0xf, 0xf, false)));
    x = fmaxf(x, __int_as_float(__builtin_amdgcn_update_dpp(ninf, __float_as_int(x), 0x118, 0xf, 0xf, false)));
    x = fmaxf(x, __int_as_float(__builtin_amdgcn_update_dpp(ninf, __float_as_int(x), 0x142, 0xa, 0xf, false)));
    x = fmaxf(x, __int_as_float(__builtin_amdgcn_update_dpp(ninf, __float_as_int(x), 0x143, 0xc, 0xf, false)));
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 63));
}
// First index holding the maximum: Python's `if score > best_score` scan over the children dict
// (mcts.py:423-428). NaN never wins (NaN > x is False); -0.0 ties +0.0. The max key on the DPP
// network, then the lowest lane holding it (all lanes invalid: lane 0).
__device__ __forceinline__ int wave_argmax_first(float s, bool valid, int lane) {
    const uint32_t key = (valid && !isnan(s)) ? score_key(s) : 0u;
    const uint32_t m = wave_max_u32(key);
    return __ffsll((unsigned long long)__ballot(key == m)) - 1;
}
// value of lane `src` (wave-uniform) to every lane
__device__ __forceinline__ int lane_bcast(int x, int src) { return __builtin_amdgcn_readlane(x, src); }
__device__ __forceinline__ float lane_bcast(float x, int src) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), src));
}

// ---- backup (mcts.py:625-640): lane j updates path node plen-1-j; `copies` sequential adds ----
// path_reg: lane i holds the i-th node of the path (root = lane 0). Returns the updated visit
// count of the root in every lane.
__device__ __forceinline__ int backup_path(Node* nodes, int path_reg, int plen, float value,
                                           int copies, int lane, bool order_before) {
    // order this wave's earlier stores to path nodes (UCB caches) before the read-modify-write
    if (order_before) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    // lane d holds the path node at depth d (the root in lane 0): each lane updates its own node
    const int nid = path_reg;
    int n_after = 0;
    if (lane < plen) {
        // sign = +1 at the leaf (depth plen - 1), then alternates toward the root
        const float sv = ((plen - 1 - lane) & 1) ? -value : value;
        Node nd = nodes[nid];
        float w = nd.w;
        for (int k = 0; k < copies; ++k) w = w + sv;
        nd.n += copies;
        nd.w = w;
        nd.c = __int_as_float(0x7fc00000);  // del cached_ucb
        nodes[nid] = nd;
        n_after = nd.n;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    return __builtin_amdgcn_readlane(n_after, 0);  // the root's lane
}

// UCB of an expanded child whose score is not cached (mcts.py:102-114); turn_c = child's turn.
// sqrt_np = sqrt_count(parent N): exactly `np.float32(math.sqrt(parent_visit_count))` as the
// reference's NumPy promotion takes it.
// np.float32(math.sqrt(n)) for a visit count n < 2^24: math.sqrt rounds the exact root to 53
// bits, the cast to 24; rounding twice through p' >= 2p + 2 bits (53 >= 50) equals rounding once
// for sqrt (Figueroa), so the correctly rounded f32 sqrt of (float)n (exact for n < 2^24) is the
// same value (-fhip-fp32-correctly-rounded-divide-sqrt; tests/test_gpu_numerics.py)
__device__ __forceinline__ float sqrt_count(int n) { return __builtin_sqrtf((float)n); }

__device__ __forceinline__ float ucb_score(const Node& c, float sqrt_np, int turn_c, float cpuct) {
    float u = cpuct * c.p;
    u = u * sqrt_np;
    u = u / (float)(1 + c.n);
    float q = c.w / (float)(c.n > 1 ? c.n : 1);
    if (turn_c != 1) q = -q;
    return q + u;
}

// Inputs of the pending expand + backup, all loaded at the head of a launch (no dependent loads:
// the leaf's meta word is kept in per-game scratch by the select that queued it).
struct ExpIn {
    int copies, plen, path_reg, e;
    uint64_t V;
    uint32_t lm;
    float val, prob, xpass;
};

template <int BS>
__device__ __forceinline__ ExpIn expand_load(const View& v, int g, int lane,
                                             const float* __restrict__ policy,
                                             const float* __restrict__ value) {
    constexpr int NSQ = Geo<BS>::NSQ, NPOL = Geo<BS>::NPOL;
    ExpIn x;
    x.copies = v.pend[g];
    x.plen = v.plen[g];
    x.path_reg = v.path[g * PATH_CAP + lane];
    x.V = v.leaf_legal[g];
    x.e = v.nexp[g];
    x.lm = v.leaf_meta[g];
    const int r = v.live ? v.row_of[g] : g;
    x.val = value[r];
    const float* row = policy + (size_t)r * NPOL;
    x.prob = lane < NSQ ? row[lane] : 0.0f;
    x.xpass = row[NSQ];
    return x;
}

// F.softmax(policy_logits, dim=1) over all S*S+1 outputs (mcts.py:596), one row per wave: lane
// s < NSQ holds logit s, every lane the pass logit; returns (lane s's probability, 0 for lanes
// >= NSQ; the pass probability). The expand's fused softmax and rvz_policy_softmax are this one
// function (the expand uses .x only: no pass child is ever created).
template <int NSQ>
__device__ __forceinline__ float2 policy_softmax(float logit, float xpass, int lane) {
    const float mx = fmaxf(wave_max_f(lane < NSQ ? logit : -INFINITY), xpass);
    const float ex = lane < NSQ ? expf(logit - mx) : 0.0f;
    const float ep = expf(xpass - mx);
    const float denom = wave_sum_f(ex) + ep;
    return make_float2(ex / denom, ep / denom);
}

// rvz_policy_softmax: one wave per row, WPB rows per workgroup
template <int BS>
__global__ __launch_bounds__(256) void k_policy_softmax(int n, const float* __restrict__ logits,
                                                        float* __restrict__ probs) {
    constexpr int NSQ = Geo<BS>::NSQ, NPOL = Geo<BS>::NPOL;
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * WPB + (threadIdx.x >> 6);
    if (r >= n) return;
    const float* row = logits + (size_t)r * NPOL;
    const float2 p = policy_softmax<NSQ>(lane < NSQ ? row[lane] : 0.0f, row[NSQ], lane);
    if (lane < NSQ) probs[(size_t)r * NPOL + lane] = p.x;
    if (lane == 0) probs[(size_t)r * NPOL + NSQ] = p.y;
}

// expand + backup of the queued leaf: _process_batch pass 2 (mcts.py:600-623) and
// MCTSNode.expand (:141-161). Returns the root's visit count after the backup (-1: nothing to
// do) and, when the expanded leaf is the root, its new meta word in *root_meta.
template <int BS>
__device__ __forceinline__ int expand_backup_phase(const View& v, int g, int lane, ExpIn x,
                                                   int is_logits, uint32_t* root_meta,
                                                   unsigned long long& ab) {
    constexpr int NSQ = Geo<BS>::NSQ, NPOL = Geo<BS>::NPOL;
    if (x.copies == 0) return -1;
    const int path_reg = lane < x.plen ? x.path_reg : 0;
    const int leaf = __builtin_amdgcn_readlane(path_reg, x.plen - 1);
    Node* nodes = v.nodes + (size_t)g * v.M;
    uint32_t* meta = v.meta + (size_t)g * v.M;
    float prob = x.prob;
    if (is_logits) prob = policy_softmax<NSQ>(prob, x.xpass, lane).x;
    {   // non-finite NN output (any of the 65 probabilities or the value): device error word
        const bool bad = !__builtin_isfinite(x.val) || !__builtin_isfinite(x.xpass) ||
                         (lane < NSQ && !__builtin_isfinite(prob));
        if (__builtin_amdgcn_ballot_w64(bad) && lane == 0) atomicOr(v.err, ERR_NN);
    }
    const int base = 1 + x.e * NSQ;
    if (base + NSQ > v.M) {
        if (lane == 0) atomicOr(v.err, ERR_POOL);
        return -1;
    }
    const uint64_t V = x.V;
    if (lane < NSQ && ((V >> lane) & 1ull)) {
        const int idx = __popcll(V & ((1ull << lane) - 1ull));
        Node c;
        c.n = 0; c.w = 0.0f; c.p = prob; c.c = __int_as_float(0x7fc00000);
        nodes[base + idx] = c;
        meta[base + idx] = meta_pack(lane, 3 - m_turn(x.lm));
    }
    const uint32_t nlm = x.lm | ((uint32_t)__popcll(V) << 11) | ((uint32_t)x.e << 18);
    if (lane == 0) {
        meta[leaf] = nlm;
        v.nexp[g] = x.e + 1;
        v.pend[g] = 0;
        if (v.memo) v.bval[(size_t)g * 2 * v.E + x.e] = x.val;   // the next search's memo
    }
    if (leaf == 0 && root_meta) *root_meta = nlm;
    // the path nodes are not among the nodes written above: no ordering needed before the RMW
    const int root_n = backup_path(nodes, path_reg, x.plen, x.val, x.copies, lane, false);
    if (v.stats) {
        // pend/plen/path/legal/nexp/leaf-meta reads, policy row + value, leaf meta w, children,
        // backup
        const unsigned long long nch = (unsigned long long)__popcll(V);
        ab += 8ull + 4ull * x.plen + 8 + 4 + 4 + 4ull * NPOL + 4 + 4 + 20ull * nch +
              32ull * x.plen + 8;
    }
    return root_n;
}

// rvz_search_skip: the last batch's leaf is not evaluated. Its evaluation would only set the
// leaf's children priors and add the value to W along the path — state the discarded tree never
// reads again — while the visit counts grow by the queued copies regardless (mcts.py:625-640), so
// N alone is backed up here and the visits, p and the move are those of the evaluated search.
__device__ __forceinline__ void backup_visits_only(const View& v, int g, int lane,
                                                   unsigned long long& ab) {
    const int copies = v.pend[g], plen = v.plen[g];
    if (copies == 0) return;
    const int path_reg = lane < plen ? v.path[g * PATH_CAP + lane] : 0;
    Node* nodes = v.nodes + (size_t)g * v.M;
    if (lane < plen) nodes[path_reg].n += copies;   // lane d: the path node at depth d
    if (lane == 0) v.pend[g] = 0;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    if (v.stats) ab += 8ull + 4ull * plen + 8ull * plen;
}

// A leaf whose position the previous search of this game already expanded (link lk: that node
// of the previous tree, kept in the other half of the pool): _process_batch pass 2 (mcts.py:
// 600-623) with that expansion's NN output instead of a new evaluation. An h2 row's outputs
// depend only on the position (test_h2_live_rows), so the priors (the softmax of the row at the
// legal squares, which are the old node's children in row-major order, exactly the squares the
// same position yields here) and the value are bitwise what the evaluator would return for this
// leaf now. The children get their own links (the old children that were expanded too); the
// value is backed up `copies` times at once, where the evaluated leaf's backup would run at the
// head of the next launch — the same point of the batch (after its terminal backups).
template <int BS>
__device__ __forceinline__ int memo_expand_backup(const View& v, int g, int lane, int leaf,
                                                  uint32_t lm, int path_reg, int plen,
                                                  uint32_t lk, int copies,
                                                  unsigned long long& ab) {
    constexpr int NSQ = Geo<BS>::NSQ;
    Node* nodes = v.nodes + (size_t)g * v.M;
    uint32_t* meta = v.meta + (size_t)g * v.M;
    const int nch = link_nchild(lk), ob = 1 + link_block(lk) * NSQ;
    // one round trip: the old children rows, the old node's value and the expansion counter
    Node oc;
    uint32_t ocm = 0;
    if (lane < nch) {
        oc = nodes[ob + lane];
        ocm = meta[ob + lane];
    }
    const float val = v.bval[(size_t)g * 2 * v.E + link_block(lk)];
    const int e = v.nexp[g];
    const int base = 1 + e * NSQ;
    if (base + NSQ > v.M) {
        if (lane == 0) atomicOr(v.err, ERR_POOL);
        return -1;
    }
    if (lane < nch) {
        Node c;
        c.n = 0; c.w = 0.0f; c.p = oc.p;
        const bool expd = m_nchild(ocm) > 0 && !m_term(ocm);
        c.c = __uint_as_float(expd ? link_pack(ob + lane, m_nchild(ocm), m_block(ocm))
                                   : LINK_NONE);
        nodes[base + lane] = c;
        meta[base + lane] = meta_pack(m_sq(ocm), 3 - m_turn(lm));
    }
    if (lane == 0) {
        meta[leaf] = lm | ((uint32_t)nch << 11) | ((uint32_t)e << 18);
        v.nexp[g] = e + 1;
        v.bval[(size_t)g * 2 * v.E + e] = val;
    }
    ab += 20ull * nch + 8 + 20ull * nch + 12 + 32ull * plen;
    // this walk's UCB-cache stores to path nodes come before the read-modify-write
    return backup_path(nodes, path_reg, plen, val, copies, lane, true);
}

// select: mcts.py:348-386 for one batch of `bsz` traversals + _process_batch pass 1 (:561-585).
// root / root_meta / root_n were loaded (or produced by the expand phase) by the caller.
template <int BS, typename XT>
__device__ __forceinline__ int select_phase(const View& v, int g, int lane, int first, int bsz,
                                             int eb,
                                             const GameS& root, uint32_t root_meta, int root_n,
                                             uint32_t carry,
                                             XT* __restrict__ leaf_x, int32_t* __restrict__ need,
                                             unsigned long long& ab,
                                             uint64_t* leaf_bits = nullptr) {
    constexpr int NSQ = Geo<BS>::NSQ;
    Node* nodes = v.nodes + (size_t)g * v.M;
    uint32_t* meta = v.meta + (size_t)g * v.M;
    if (first) {  // new root (mcts.py:334-341): prior 1.0, turn = side to move
        root_meta = meta_pack(0, root.side);
        root_n = 0;
        // memo: this search's blocks go to the half the previous tree (where the carried node
        // lives) does not use; without a carried node, half 0
        const int half = (v.memo && link_ok(carry) && (link_node(carry) - 1) / NSQ < v.E) ? 1 : 0;
        if (lane == 0) {
            Node r;
            r.n = 0; r.w = 0.0f; r.p = 1.0f; r.c = __int_as_float(0x7fc00000);
            nodes[0] = r;
            meta[0] = root_meta;
            v.nexp[g] = half * v.E;
        }
        const uint64_t rl = root.over ? 0ull : legal_wave<BS>(mine(root), theirs(root), lane);
        if (lane == 0) v.root_legal[g] = rl;
        ab += 20 + 8;
    }
    ab += 32 + 8;  // game state, root meta + N
    int copies = 0, plen = 0, path_reg = 0;
    if (!root.over) {
        int remaining = bsz;
        for (;;) {
            WALK_STAT(0, 1);
            WT_NOW(tw0);
            GameS sim = root;
            int depth = 0, node = 0, parent_n = root_n;
            uint32_t m = root_meta;
            // memo link of the node the walk ends on (the root's: the carried node)
            uint32_t lk = first ? carry : LINK_NONE;
            path_reg = 0;  // lane 0 holds the root
            // per level d (in lane d): the chosen child's index, its turn for scoring, the best
            // other child's score and index (-1: none) — the terminal fast path below
            int fp_ci = 0, fp_b = -1, fp_turn = 0;
            float fp_sb = 0.0f;
            bool truncated = false;
            // the move of level d (lane d): replayed on `sim` only if the walk ends on a leaf
            // that needs the position (a known terminal does not)
            int fp_sq = 0;
            for (;;) {
                const int nch = m_nchild(m);
                if (m_term(m) || nch == 0) break;  // while node.expanded() and not terminal
                const int base = 1 + m_block(m) * NSQ;
                // one round trip per level: the children's node rows and meta words together
                Node c;
                uint32_t cm = 0;
                if (lane < nch) {
                    c = nodes[base + lane];
                    cm = meta[base + lane];
                } else {
                    c.n = 0; c.w = 0.0f; c.p = 0.0f; c.c = 0.0f;
                }
                float score = 0.0f;
                bool wrote = false;
                if (lane < nch) {
                    if (c.n == 0) {
                        score = INFINITY;
                    } else if (!isnan(c.c)) {
                        score = c.c;
                    } else {
                        const float sq_np = sqrt_count(parent_n);
                        score = ucb_score(c, sq_np, 3 - m_turn(m), v.cpuct);
                        nodes[base + lane].c = score;
                        wrote = true;
                    }
                }
                WALK_STAT(1, 1);
                const int ci = wave_argmax_first(score, lane < nch, lane);
                const int bsib = wave_argmax_first(score, lane < nch && lane != ci, lane);
                const float sbs = lane_bcast(score, bsib);
                const int turn_c = 3 - m_turn(m);
                if (v.stats) ab += 16ull * nch + 4ull * nch + 4ull * __popcll(__ballot(wrote));
                node = base + ci;
                m = (uint32_t)lane_bcast((int)cm, ci);
                parent_n = lane_bcast(c.n, ci);
                if (v.memo) lk = (uint32_t)lane_bcast(__float_as_int(c.c), ci);
                ++depth;
                if (depth >= PATH_CAP) {  // unreachable when ceil(sims/batch) <= 64 (checked)
                    if (lane == 0) atomicOr(v.err, ERR_PATH);
                    depth = PATH_CAP - 1;
                    truncated = true;
                    break;
                }
                if (lane == depth) {
                    path_reg = node;
                    fp_sq = m_sq(m);
                    fp_ci = ci;
                    fp_b = nch > 1 ? bsib : -1;
                    fp_sb = sbs;
                    fp_turn = turn_c;
                }
            }
            WT_ADD(1, tw0);
            if (m_term(m)) {  // known terminal: back up its value at once (mcts.py:364-366)
                WT_NOW(tb0);
                root_n = backup_path(nodes, path_reg, depth + 1, m_tv(m), 1, lane, true);
                WALK_STAT(2, 1);
                WT_ADD(2, tb0);
                ab += 32ull * (depth + 1);
                if (--remaining == 0) break;
                if (truncated) continue;
                // Fast path for the next traversals while they provably reach the same terminal.
                // A backup invalidates only the path nodes' cached scores (mcts.py:639-640), so
                // every other child on the path keeps the score this walk saw; the next walk
                // takes the same child at level d iff the path child's fresh score (the reference
                // formula on its backed-up N, W and its parent's N) beats the best other child
                // under the first-index tie-break. Register copies of the path nodes replace the
                // re-walk and its backup; the path is written back once (N, W, cache invalid)
                // before the walk resumes at the first divergence or the batch ends.
                WT_NOW(tf0);
                const float tv = m_tv(m);
                Node pn;
                if (lane <= depth) pn = nodes[path_reg];
                int fn = lane <= depth ? pn.n : 0;
                float fw = lane <= depth ? pn.w : 0.0f;
                const float fpr = lane <= depth ? pn.p : 0.0f;
                int hits = 0;
                for (;;) {
                    const int par_n = __shfl_up(fn, 1);
                    bool hold = true;
                    if (lane >= 1 && lane <= depth && fp_b >= 0) {
                        Node cn;
                        cn.n = fn; cn.w = fw; cn.p = fpr; cn.c = 0.0f;
                        const float sc = ucb_score(cn, sqrt_count(par_n), fp_turn,
                                                   v.cpuct);
                        const uint32_t ks = score_key(sc), kb = score_key(fp_sb);
                        hold = ks > kb || (ks == kb && fp_ci < fp_b);
                    }
                    if (__ballot(!hold) != 0ull) break;
                    if (lane <= depth) {   // _backpropagate_path of the same terminal value
                        fw = fw + (((depth - lane) & 1) ? -tv : tv);
                        fn += 1;
                    }
                    ++hits;
                    WALK_STAT(3, 1);
                    if (--remaining == 0) break;
                }
                if (hits) {
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
                    if (lane <= depth) {
                        Node nd;
                        nd.n = fn; nd.w = fw; nd.p = fpr; nd.c = __int_as_float(0x7fc00000);
                        nodes[path_reg] = nd;
                    }
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
                    root_n = __builtin_amdgcn_readlane(fn, 0);
                }
                ab += 32ull * (depth + 1);
                WT_ADD(3, tf0);
                if (remaining == 0) break;
                continue;
            }
            if (v.memo && link_ok(lk) && !truncated) {
                // the previous search evaluated this position: expand it from that output, no
                // NN row (the position has legal moves, so it is not terminal)
                const int rn = memo_expand_backup<BS>(v, g, lane, node, m, path_reg, depth + 1,
                                                      lk, remaining, ab);
                if (rn >= 0) root_n = rn;
                break;
            }
            WT_NOW(tl0);
            // the leaf's position: the path's moves on the root's game (a truncated path, an
            // error already flagged, replays its first PATH_CAP - 1 moves)
            for (int d = 1; d <= depth; ++d)
                make_move_wave<BS>(sim, __builtin_amdgcn_readlane(fp_sq, d), lane);
            // pass 1: valid moves of the leaf's simulated game
            const uint64_t V = legal_wave<BS>(mine(sim), theirs(sim), lane);
            if (V == 0ull) {  // terminal, BLACK-absolute value from get_winner() (mcts.py:567-579)
                const int w = sim.over ? sim.winner : -1;
                const uint32_t code = w == 1 ? 1u : (w == 2 ? 2u : 0u);
                if (lane == 0) meta[node] = m | (1u << 8) | (code << 9);
                WALK_STAT(4, 1);
                backup_path(nodes, path_reg, depth + 1, w == 1 ? 1.0f : (w == 2 ? -1.0f : 0.0f),
                            remaining, lane, true);
                ab += 4 + 32ull * (depth + 1);
                break;
            }
            // queue `remaining` identical copies for the NN: encode get_canonical_state() planes
            copies = remaining;
            plen = depth + 1;
            // compacted batch: the next free row of batch eb (one atomic per live game)
            int r = g;
            if (v.live) {   // striped counters: at most STRIPE contending waves per address
                const int s = g / RVZ_LIVE_STRIPE;
                if (lane == 0)
                    r = s * RVZ_LIVE_STRIPE +
                        atomicAdd(v.live + ((size_t)eb * v.NS + s) * RVZ_LIVE_PITCH, 1);
                r = __builtin_amdgcn_readlane(r, 0);
                if (lane == 0) v.row_of[g] = r;
            }
            if (leaf_bits) {   // k_play: the planes as bitboards (P, O, V) in LDS
                if (lane == 0) {
                    leaf_bits[0] = mine(sim);
                    leaf_bits[1] = theirs(sim);
                    leaf_bits[2] = V;
                }
            } else if (lane < NSQ) {
                XT* row = leaf_x + (size_t)r * 3 * NSQ;
                const uint64_t P = mine(sim), O = theirs(sim);
                row[lane] = (XT)(float)((P >> lane) & 1ull);
                row[NSQ + lane] = (XT)(float)((O >> lane) & 1ull);
                row[2 * NSQ + lane] = (XT)(float)((V >> lane) & 1ull);
            }
            if (lane < plen) v.path[g * PATH_CAP + lane] = path_reg;
            if (lane == 0) {
                v.leaf_legal[g] = V;
                v.leaf_meta[g] = m;
            }
            WT_ADD(4, tl0);
            ab += 3ull * NSQ * sizeof(XT) + 4ull * plen + 12;
            break;
        }
    }
    if (lane == 0) {
        need[g] = copies;
        v.pend[g] = copies;
        v.plen[g] = plen;
    }
    ab += 12;
    return copies;   // the queued copies of the batch's NN row (0: no row)
}

// One search round: the previous batch's expand + backup (when a submit is pending), then the
// next batch's selection, in one launch (one wave per game). Every load that does not depend on
// another is issued at the head.
// RVZ_STEP_WPE (experiments): amdgpu_waves_per_eu cap of k_step (e.g. 7 = 72 VGPRs)
#ifdef RVZ_STEP_WPE
#define RVZ_STEP_ATTR __attribute__((amdgpu_waves_per_eu(RVZ_STEP_WPE)))
#else
#define RVZ_STEP_ATTR
#endif
template <int BS, typename XT>
__global__ __launch_bounds__(256) RVZ_STEP_ATTR void k_step(View v, int expand, const float* __restrict__ policy,
                                              int is_logits, const float* __restrict__ value,
                                              int first, int bsz, int eb,
                                              XT* __restrict__ leaf_x,
                                              int32_t* __restrict__ need) {
    const int lane = threadIdx.x & 63;
    const int g = blockIdx.x * WPB + (threadIdx.x >> 6);
    if (g >= v.G) return;
    const GameS root = load_game(v, g);
    uint32_t root_meta = 0, carry = LINK_NONE;
    int root_n = 0;
    if (!first) {
        root_meta = v.meta[(size_t)g * v.M];
        root_n = v.nodes[(size_t)g * v.M].n;
    } else if (v.memo) {
        carry = v.carry[g];
    }
    unsigned long long ab_e = 0, ab_s = 0;
    WT_NOW(te0);
    if (expand) {
        const ExpIn x = expand_load<BS>(v, g, lane, policy, value);
        const int rn = expand_backup_phase<BS>(v, g, lane, x, is_logits, &root_meta, ab_e);
        if (rn >= 0) root_n = rn;
    }
    WT_ADD(0, te0);
    select_phase<BS, XT>(v, g, lane, first, bsz, eb, root, root_meta, root_n, carry, leaf_x, need,
                         ab_s);
    if (v.stats && lane == 0) v.stats[g] += ab_s + ab_e;  // per-game slot: no contention
}

template <int BS>
__global__ __launch_bounds__(256) void k_expand_backup(View v, int mode,
                                                       const float* __restrict__ policy,
                                                       int is_logits,
                                                       const float* __restrict__ value) {
    const int lane = threadIdx.x & 63;
    const int g = blockIdx.x * WPB + (threadIdx.x >> 6);
    if (g >= v.G) return;
    unsigned long long ab = 0;
    if (mode == 2) {
        backup_visits_only(v, g, lane, ab);
    } else {
        const ExpIn x = expand_load<BS>(v, g, lane, policy, value);
        expand_backup_phase<BS>(v, g, lane, x, is_logits, nullptr, ab);
    }
    if (v.stats && lane == 0) v.stats[2 * (size_t)v.G + g] += ab;
}

// Dense visit count of square `lane` at the root: the root's children are the set bits of the
// search root's legal mask in ascending order (expand inserts them row-major).
template <int BS>
__device__ __forceinline__ int root_visits(const View& v, int g, int lane) {
    constexpr int NSQ = Geo<BS>::NSQ;
    const Node* nodes = v.nodes + (size_t)g * v.M;
    const uint32_t m0 = v.meta[(size_t)g * v.M];
    const uint64_t V = v.root_legal[g];
    const int nch = m_nchild(m0);
    if (nch == 0 || lane >= NSQ) return 0;
    if (!((V >> lane) & 1ull)) return 0;
    const int idx = __popcll(V & ((1ull << lane) - 1ull));
    return nodes[1 + m_block(m0) * NSQ + idx].n;
}

template <int BS>
__global__ __launch_bounds__(256) void k_visits(View v, int32_t* __restrict__ out) {
    constexpr int NSQ = Geo<BS>::NSQ, NPOL = Geo<BS>::NPOL;
    const int lane = threadIdx.x & 63;
    const int g = blockIdx.x * WPB + (threadIdx.x >> 6);
    if (g >= v.G) return;
    const int n = root_visits<BS>(v, g, lane);
    if (lane < NSQ) out[(size_t)g * NPOL + lane] = n;
    if (lane == 0) out[(size_t)g * NPOL + NSQ] = 0;  // no pass child is ever created
}

// numpy `arr ** e` for float64 (fast_scalar_power paths, else the correctly rounded power; NumPy's
// general power is host-dependent, csrc/rvz_pow.hip.h)
__device__ __forceinline__ double np_power(double x, double e) {
    if (e == 1.0) return x;
    if (e == 2.0) return x * x;
    if (e == 0.5) return sqrt(x);
    if (e == -1.0) return 1.0 / x;
    if (e == 0.0) return 1.0;
    return rvz_pow::pow_cr(x, e);
}

// act for one game (one wave): the search's pending expand (expand 1) or visit-count backup
// (expand 2), then get_action_probs' tail and the move; returns the sampled index (-2: the game
// was over). s: NPOL + 7 doubles of this wave's LDS.
template <int BS>
__device__ __forceinline__ int act_game(const View& v, int g, int lane, double* s, int expand,
                                        const float* __restrict__ policy, int is_logits,
                                        const float* __restrict__ value, double temperature,
                                        const double* __restrict__ uo, int apply,
                                        int32_t* __restrict__ out_idx, double* __restrict__ out_p,
                                        bool* over_after = nullptr) {
    constexpr int NSQ = Geo<BS>::NSQ, NPOL = Geo<BS>::NPOL;
    constexpr int NMAIN = NPOL - NPOL % 8;
    unsigned long long ab = 0;
    if (expand == 1) {
        const ExpIn x = expand_load<BS>(v, g, lane, policy, value);
        expand_backup_phase<BS>(v, g, lane, x, is_logits, nullptr, ab);
    } else if (expand == 2) {
        backup_visits_only(v, g, lane, ab);
    }
    GameS gm = load_game(v, g);
    double* prow = out_p + (size_t)g * NPOL;
    if (gm.over) {
        if (lane < NSQ) prow[lane] = 0.0;
        if (lane == 0) {
            prow[NSQ] = 0.0;
            out_idx[g] = -2;
            if (v.memo) v.carry[g] = LINK_NONE;
            if (v.stats) v.stats[(size_t)v.G + g] += ab + 32 + 8ull * NPOL + 4;
        }
        if (over_after) *over_after = true;
        return -2;
    }
    const int n = root_visits<BS>(v, g, lane);
    const int total = wave_sum_i(n);
    double p = (lane < NSQ && total > 0) ? (double)n / (double)total : 0.0;
    double ppass = 0.0;
    if (temperature > 0.0 && __any(p != 0.0)) {
        const double ex = 1.0 / temperature;
        const double t = lane < NSQ ? np_power(p, ex) : 0.0;
        const double tp = np_power(0.0, ex);
        // np.sum in numpy's pairwise order: 8 accumulators over the first NMAIN entries, then tail
        if (lane < NSQ) s[lane] = t;
        if (lane == 0) s[NSQ] = tp;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        __builtin_amdgcn_wave_barrier();
        double r = 0.0;
        if (lane < 8) {
            r = s[lane];
            for (int i = 8 + lane; i < NMAIN; i += 8) r += s[i];
        }
        const double r0 = __shfl(r, 0), r1 = __shfl(r, 1), r2 = __shfl(r, 2), r3 = __shfl(r, 3);
        const double r4 = __shfl(r, 4), r5 = __shfl(r, 5), r6 = __shfl(r, 6), r7 = __shfl(r, 7);
        double sum = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
        for (int i = NMAIN; i < NPOL; ++i) sum += s[i];
        p = t / sum;
        ppass = tp / sum;
        __builtin_amdgcn_wave_barrier();
    }
    const bool all_zero = !__any(lane < NSQ && p != 0.0) && ppass == 0.0;
    if (lane < NSQ) s[lane] = p;
    if (lane == 0) s[NSQ] = ppass;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
    int idx = 0;
    if (temperature == 0.0 || all_zero) {  // np.argmax: first maximum
        if (lane == 0) {
            double best = s[0];
            for (int i = 1; i < NPOL; ++i)
                if (s[i] > best) { best = s[i]; idx = i; }
        }
    } else {  // np.random.choice(NPOL, p=p): cumsum, /= last, searchsorted(u, 'right')
        double u;
        if (uo) {
            u = uo[g];
        } else {
            const int pos = v.rng_pos[g];
            if (pos >= RNG_DRAWS) {
                if (lane == 0) atomicOr(v.err, ERR_RNG);
                u = 0.0;
            } else {
                u = v.rng_u[(size_t)g * RNG_DRAWS + pos];
            }
            if (lane == 0) v.rng_pos[g] = pos + 1;
        }
        if (lane == 0) {
            double acc = 0.0;  // cdf[-1]: the same sequential adds as p.cumsum()
            for (int i = 0; i < NPOL; ++i) acc += s[i];
            const double last = acc;
            acc = 0.0;
            for (int i = 0; i < NPOL; ++i) {
                acc += s[i];
                if (acc / last <= u) idx = i + 1;  // count of cdf entries <= u
            }
        }
    }
    idx = __shfl(idx, 0);
    if (lane < NSQ) prow[lane] = p;
    if (lane == 0) {
        prow[NSQ] = ppass;
        out_idx[g] = idx;
    }
    if (apply) {
        make_move_wave<BS>(gm, idx == NSQ ? -1 : idx, lane);  // (-1, -1) for the pass index
        if (lane == 0) store_game(v, g, gm);
    }
    if (over_after) *over_after = gm.over != 0;
    if (v.memo && lane == 0) {
        // the child the move went to (its position is the next search's root), if this search
        // expanded it: the next search's root takes that expansion's NN output (memo_expand_backup)
        uint32_t cl = LINK_NONE;
        const uint32_t m0 = v.meta[(size_t)g * v.M];
        const uint64_t V = v.root_legal[g];
        if (apply && idx < NSQ && m_nchild(m0) > 0 && ((V >> idx) & 1ull)) {
            const int c = 1 + m_block(m0) * NSQ + __popcll(V & ((1ull << idx) - 1ull));
            const uint32_t cm = v.meta[(size_t)g * v.M + c];
            if (m_nchild(cm) > 0 && !m_term(cm)) cl = link_pack(c, m_nchild(cm), m_block(cm));
        }
        v.carry[g] = cl;
    }
    if (v.stats && lane == 0)  // state r/(w), root meta + children N, p row + idx, rng
        v.stats[(size_t)v.G + g] += ab + 32ull + (apply ? 32 : 0) + 12 +
                                    4ull * m_nchild(v.meta[(size_t)g * v.M]) + 8ull * NPOL + 4 + 16;
    return idx;
}

#ifndef RVZ_ACT_WPE
#define RVZ_ACT_WPE 6
#endif
// act: mcts.py:656-692 + self_play.py:98 (make_move of the sampled action); optionally preceded
// by the last batch's pending expand + backup.
template <int BS>
// 8x8: <= 80 VGPRs (6 waves per SIMD), so a k_act wave fits on a SIMD beside two trunk waves
// (2 x 216); the 6x6 form would spill under that cap
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(BS == 8 ? RVZ_ACT_WPE : 1))) void k_act(View v, int expand, const float* __restrict__ policy,
                                             int is_logits, const float* __restrict__ value,
                                             double temperature, const double* __restrict__ uo,
                                             int apply, int32_t* __restrict__ out_idx,
                                             double* __restrict__ out_p) {
    constexpr int NPOL = Geo<BS>::NPOL;
    __shared__ double sp[WPB][NPOL + 7];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int g = blockIdx.x * WPB + wid;
    if (g >= v.G) return;
    // the search's leaf batches are all consumed (their NN calls precede this launch); the rows
    // of a skipped last batch (expand == 2, rvz_search_skip) were handed out but not evaluated
    if (v.live && lane == 0) {
        const int counted = expand == 2 ? (v.E - 1) * v.NS : v.E * v.NS;
        for (int i = g; i < v.E * v.NS; i += v.G) {
            const int c = v.live[(size_t)i * RVZ_LIVE_PITCH];
            if (c && i < counted) atomicAdd(v.live_total, (unsigned long long)c);
            v.live[(size_t)i * RVZ_LIVE_PITCH] = 0;
        }
    }
    act_game<BS>(v, g, lane, sp[wid], expand, policy, is_logits, value, temperature, uo, apply,
                 out_idx, out_p);
}

// reset: new game (board.py:25-39) + np.random.seed(seed) random_sample() stream.
// a fresh game g seeded with `seed` (np.random.seed semantics): MT19937 init, its first draws,
// the start position (one wave; k is the wave's 624-word key scratch in LDS)
template <int BS>
__device__ __forceinline__ void reset_game(const View& v, int g, int lane, uint32_t seed,
                                           uint32_t* k) {
    if (lane == 0) {  // mt19937_seed (init_genrand): inherently sequential
        uint32_t sd = seed;
        for (int pos = 0; pos < 624; ++pos) {
            k[pos] = sd;
            sd = 1812433253u * (sd ^ (sd >> 30)) + (uint32_t)(pos + 1);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
    // First generation: words 0..127 only need the initial key (i + 397 < 624 for i < 227).
    auto word = [&](int i) -> uint32_t {
        const uint32_t y = (k[i] & 0x80000000u) | (k[i + 1] & 0x7fffffffu);
        uint32_t x = k[i + 397] ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
        x ^= (x >> 11);
        x ^= (x << 7) & 0x9d2c5680u;
        x ^= (x << 15) & 0xefc60000u;
        x ^= (x >> 18);
        return x;
    };
    const uint32_t a = word(2 * lane) >> 5, b = word(2 * lane + 1) >> 6;
    v.rng_u[(size_t)g * RNG_DRAWS + lane] = ((double)a * 67108864.0 + (double)b) / 9007199254740992.0;
    if (lane == 0) {
        GameS st;
        st.black = Geo<BS>::START_BLACK;
        st.white = Geo<BS>::START_WHITE;
        st.side = 1; st.over = 0; st.winner = -1; st.passed = 0;
        store_game(v, g, st);
        v.rng_pos[g] = 0;
        v.pend[g] = 0;
        v.carry[g] = LINK_NONE;   // a new game: nothing to carry into its first search
    }
}

template <int BS>
__global__ __launch_bounds__(256) void k_reset(View v, const uint32_t* __restrict__ seeds,
                                               const uint8_t* __restrict__ mask) {
    __shared__ uint32_t key[WPB][624];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int g = blockIdx.x * WPB + wid;
    if (g >= v.G) return;
    if (mask && !mask[g]) return;
    reset_game<BS>(v, g, lane, seeds[g], key[wid]);
}

// The self-play driver's per-ply bookkeeping in one launch (SelfPlayRunner, self_play.py:80-101
// run back to back): plies[g] += (idx[g] >= 0) (a move was committed); when `reset`, a game that
// just ended counts in done[g], takes its slot's next seed (seeds[g] += stride) and restarts from
// the start position with it. Per-game counters: no contended atomics; the totals are summed
// when read.
template <int BS>
__global__ __launch_bounds__(256) void k_autoreset(View v, const int32_t* __restrict__ idx,
                                                   int64_t* __restrict__ seeds, int64_t stride,
                                                   int64_t* __restrict__ plies,
                                                   int64_t* __restrict__ done, int reset) {
    __shared__ uint32_t key[WPB][624];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int g = blockIdx.x * WPB + wid;
    if (g >= v.G) return;
    if (lane == 0 && idx[g] >= 0) plies[g] += 1;
    if (!reset || !v.status[4 * g + 1]) return;
    int64_t sd = 0;
    if (lane == 0) {
        done[g] += 1;
        sd = seeds[g] + stride;
        seeds[g] = sd;
    }
    sd = __shfl(sd, 0);
    reset_game<BS>(v, g, lane, (uint32_t)(sd & 0xFFFFFFFFll), key[wid]);
}

#include "rvz_play.hip.h"
// (The team-specialised fused kernel k_play12 of round 4 — measured 4% behind k_play, DESIGN
// §8.6 — is kept as tools/patches/play12_teams.patch, not in the product library.)

// ---- board kernels on caller arrays (one thread per board) --------------------------------------
template <int BS>
__global__ void k_board_legal(int n, const uint64_t* __restrict__ black,
                              const uint64_t* __restrict__ white, const int32_t* __restrict__ status,
                              uint64_t* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int side = status[4 * i];
    const uint64_t P = side == 1 ? black[i] : white[i], O = side == 1 ? white[i] : black[i];
    out[i] = legal<BS>(P, O);
}

template <int BS>
__global__ void k_board_apply(int n, uint64_t* __restrict__ black, uint64_t* __restrict__ white,
                              int32_t* __restrict__ status, const int32_t* __restrict__ sq,
                              int32_t* __restrict__ ok) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    GameS s;
    s.black = black[i];
    s.white = white[i];
    const int4 st = reinterpret_cast<const int4*>(status)[i];
    s.side = st.x; s.over = st.y; s.winner = st.z; s.passed = st.w;
    const bool r = make_move<BS>(s, sq[i]);
    if (r) {
        black[i] = s.black;
        white[i] = s.white;
        reinterpret_cast<int4*>(status)[i] = make_int4(s.side, s.over, s.winner, s.passed);
    }
    if (ok) ok[i] = r ? 1 : 0;
}

template <int BS>
__global__ void k_board_canonical(int n, const uint64_t* __restrict__ black,
                                  const uint64_t* __restrict__ white,
                                  const int32_t* __restrict__ status, float* __restrict__ out) {
    constexpr int NSQ = Geo<BS>::NSQ;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = t / NSQ, s = t % NSQ;
    if (i >= n) return;
    const int side = status[4 * i];
    const uint64_t P = side == 1 ? black[i] : white[i], O = side == 1 ? white[i] : black[i];
    const uint64_t V = legal<BS>(P, O);
    float* row = out + (size_t)i * 3 * NSQ;
    row[s] = (float)((P >> s) & 1ull);
    row[NSQ + s] = (float)((O >> s) & 1ull);
    row[2 * NSQ + s] = (float)((V >> s) & 1ull);
}

}  // namespace

// =================================================================================================
// host side
// =================================================================================================
struct rvz_engine {
    rvz_config cfg;
    int BS, NSQ, NPOL, E, M;
    hipStream_t stream = nullptr;
    int next_batch = 0;  // batches issued in the current search
    int32_t* live_buf = nullptr;    // rvz_search_compact: [E] live counts + [G] row map + total
    unsigned long long* live_total = nullptr;
    int live_dirty = 0;             // a k_step counted since the last k_act zeroed the counts
    int searching = 0;
    // a submitted batch whose expand + backup runs at the start of the next launch (k_step/k_act)
    int pending = 0;
    const float* pend_policy = nullptr;
    const float* pend_value = nullptr;
    int pend_is_logits = 0;
    int64_t counters[2] = {0, 0};
    View v;
    unsigned long long* stats_buf = nullptr;
    // launch timing (rvz_timing_enable): HIP event pairs around k_step / k_act on the stream
    int timing = 0;
    std::vector<hipEvent_t> ev_pool;
    size_t ev_used = 0;
    std::vector<std::pair<int, size_t>> ev_marks;  // (kind 0 = k_step, 1 = k_act, first event)
    std::vector<void*> allocs;
    std::string err;
    // rvz_play_table: the cross-game NN-output table (tab null: off)
    unsigned long long* tab = nullptr;
    unsigned* tclaim = nullptr;
    unsigned* tgen = nullptr;
    int64_t tslots = 0;
    int tmaxd = 0;
    const void* tab_blob = nullptr;   // the weight blob the current generation's rows came from
    // rvz_play_gate: the per-XCD pass gate of the 10x128 k_play form (fraction < 0: the default)
    double gate_frac = -1.0, gate_us = 0.0, gate_late_us = 0.0;
};

static thread_local std::string g_create_error;

#define RVZ_HIP(call, e)                                                                   \
    do {                                                                                   \
        hipError_t _s = (call);                                                            \
        if (_s != hipSuccess) {                                                            \
            (e)->err = std::string(#call) + ": " + hipGetErrorString(_s);                  \
            return RVZ_EHIP;                                                               \
        }                                                                                  \
    } while (0)

static int launch_check(rvz_engine* e, const char* what) {
    hipError_t s = hipGetLastError();
    if (s != hipSuccess) {
        e->err = std::string(what) + ": " + hipGetErrorString(s);
        return RVZ_EHIP;
    }
    e->counters[1] += 1;
    return RVZ_OK;
}

static int grid_games(int G) { return (G + WPB - 1) / WPB; }

// Stream-ordered 32-bit fill as a kernel of our own instead of hipMemsetAsync: inside a captured
// HIP graph a memset node's replays were seen to leave device words of the filled buffer
// holding a 64-bit address (tools/diag_stagger.py: rvz_play's queue words after the second replay
// of a 60-ply graph), after which the queue's task counter never reset. A kernel node has no
// such problem, and costs one ~2 us launch.
__global__ __launch_bounds__(256) void k_fill32(uint32_t* __restrict__ p, uint32_t v, size_t n) {
    for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        p[i] = v;
}

// a new table generation (new weights): every slot of an older generation reads as empty
__global__ void k_table_bump(unsigned* gen) {
    if (threadIdx.x == 0) atomicAdd(gen, 1u);
}

static int table_bump(rvz_engine* e) {
    if (!e->tgen) return RVZ_OK;
    hipLaunchKernelGGL(k_table_bump, dim3(1), dim3(64), 0, e->stream, e->tgen);
    RVZ_HIP(hipGetLastError(), e);
    return RVZ_OK;
}

static void table_free(rvz_engine* e) {
    for (void* p : {(void*)e->tab, (void*)e->tclaim, (void*)e->tgen})
        if (p) (void)hipFree(p);
    e->tab = nullptr;
    e->tclaim = nullptr;
    e->tgen = nullptr;
    e->tslots = 0;
    e->tab_blob = nullptr;
}

static hipError_t fill32_async(void* p, uint32_t v, size_t n, hipStream_t st) {
    if (n == 0) return hipSuccess;
    size_t blocks = (n + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    hipLaunchKernelGGL(k_fill32, dim3((unsigned)blocks), dim3(256), 0, st,
                       static_cast<uint32_t*>(p), v, n);
    return hipGetLastError();
}

// Timing events: no system-scope fence (a fenced record writes back and invalidates the caches,
// which would both slow the timed kernel and inflate the interval).
static hipEvent_t timing_event(rvz_engine* e) {
    if (e->ev_used == e->ev_pool.size()) {
        hipEvent_t ev = nullptr;
        if (hipEventCreateWithFlags(&ev, hipEventDisableSystemFence) != hipSuccess) return nullptr;
        e->ev_pool.push_back(ev);
    }
    return e->ev_pool[e->ev_used++];
}

static void timing_begin(rvz_engine* e, int kind) {
    if (!e->timing) return;
    hipEvent_t a = timing_event(e), b = timing_event(e);
    if (!a || !b) { e->timing = 0; return; }
    e->ev_marks.push_back({kind, e->ev_used - 2});
    (void)hipEventRecord(a, e->stream);
}

static void timing_end(rvz_engine* e) {
    if (!e->timing || e->ev_marks.empty()) return;
    (void)hipEventRecord(e->ev_pool[e->ev_marks.back().second + 1], e->stream);
}

template <typename T>
static T* dalloc(rvz_engine* e, size_t count) {
    void* p = nullptr;
    if (hipMalloc(&p, count * sizeof(T)) != hipSuccess) p = nullptr;
    e->allocs.push_back(p);
    return static_cast<T*>(p);
}

extern "C" {

int rvz_version(void) { return 1; }

const char* rvz_last_error(const rvz_engine* e) {
    return e ? e->err.c_str() : g_create_error.c_str();
}

int rvz_create(const rvz_config* cfg, rvz_engine** out) {
    if (!cfg || !out) { g_create_error = "null argument"; return RVZ_EINVAL; }
    *out = nullptr;
    const int bs = cfg->board_size;
    if (bs != 8 && bs != 6) { g_create_error = "board_size must be 8 or 6"; return RVZ_EINVAL; }
    if (cfg->n_games <= 0 || cfg->num_simulations <= 0 || cfg->batch_size <= 0) {
        g_create_error = "n_games, num_simulations and batch_size must be positive";
        return RVZ_EINVAL;
    }
    const int E = (cfg->num_simulations + cfg->batch_size - 1) / cfg->batch_size;
    if (E > PATH_CAP) {
        g_create_error = "ceil(num_simulations / batch_size) must be <= 64";
        return RVZ_EINVAL;
    }
    if (cfg->leaf_dtype != RVZ_LEAF_F32 && cfg->leaf_dtype != RVZ_LEAF_BF16) {
        g_create_error = "leaf_dtype must be RVZ_LEAF_F32 or RVZ_LEAF_BF16";
        return RVZ_EINVAL;
    }
    if (hipSetDevice(cfg->device) != hipSuccess) { g_create_error = "hipSetDevice failed"; return RVZ_EHIP; }
    rvz_engine* e = new rvz_engine();
    e->cfg = *cfg;
    e->BS = bs;
    e->NSQ = bs * bs;
    e->NPOL = e->NSQ + 1;
    e->E = E;
    // root + E expansion blocks; rvz_search_memo(on) grows the pool to two halves of E blocks
    // (the memo's two trees) the first time it is enabled, so memo-off engines hold one tree
    e->M = 1 + E * e->NSQ;
    e->v.E = E;
    e->v.NS = (cfg->n_games + RVZ_LIVE_STRIPE - 1) / RVZ_LIVE_STRIPE;
    e->v.live = nullptr;
    e->v.row_of = nullptr;
    e->v.live_total = nullptr;
    const int G = cfg->n_games;
    View& v = e->v;
    v.G = G;
    v.M = e->M;
    v.cpuct = (float)cfg->c_puct;
    v.black = dalloc<uint64_t>(e, G);
    v.white = dalloc<uint64_t>(e, G);
    v.status = dalloc<int32_t>(e, (size_t)G * 4);
    v.nodes = dalloc<Node>(e, (size_t)G * e->M);
    v.meta = dalloc<uint32_t>(e, (size_t)G * e->M);
    v.path = dalloc<int32_t>(e, (size_t)G * PATH_CAP);
    v.pend = dalloc<int32_t>(e, G);
    v.plen = dalloc<int32_t>(e, G);
    v.leaf_legal = dalloc<uint64_t>(e, G);
    v.root_legal = dalloc<uint64_t>(e, G);
    v.leaf_meta = dalloc<uint32_t>(e, G);
    v.nexp = dalloc<int32_t>(e, G);
    v.rng_u = dalloc<double>(e, (size_t)G * RNG_DRAWS);
    v.rng_pos = dalloc<int32_t>(e, G);
    v.err = dalloc<int32_t>(e, 1);
    v.memo = 0;
    v.carry = dalloc<uint32_t>(e, G);
    v.bval = dalloc<float>(e, (size_t)G * 2 * E);
    e->stats_buf = dalloc<unsigned long long>(e, 3 * (size_t)G);
    v.stats = nullptr;
    for (void* p : e->allocs)
        if (!p) { g_create_error = "hipMalloc failed (out of device memory?)"; rvz_destroy(e); return RVZ_ENOMEM; }
    hipError_t s = hipMemset(v.err, 0, sizeof(int32_t));
    s = s == hipSuccess ? hipMemset(v.pend, 0, sizeof(int32_t) * G) : s;
    s = s == hipSuccess ? hipMemset(v.rng_pos, 0, sizeof(int32_t) * G) : s;
    s = s == hipSuccess ? hipMemset(v.meta, 0, sizeof(uint32_t) * (size_t)G * e->M) : s;
    s = s == hipSuccess ? hipMemset(v.root_legal, 0, sizeof(uint64_t) * G) : s;
    s = s == hipSuccess ? hipMemset(v.leaf_meta, 0, sizeof(uint32_t) * G) : s;
    s = s == hipSuccess ? hipMemset(v.path, 0, sizeof(int32_t) * G * PATH_CAP) : s;
    s = s == hipSuccess ? hipMemsetD32(v.carry, LINK_NONE, G) : s;
    if (s == hipSuccess) s = hipDeviceSynchronize();
    if (s != hipSuccess) {
        g_create_error = std::string("device init: ") + hipGetErrorString(s);
        rvz_destroy(e);
        return RVZ_EHIP;
    }
    *out = e;
    // every game starts at the start position with seed = game index until rvz_env_reset
    std::vector<uint32_t> seeds(G);
    for (int g = 0; g < G; ++g) seeds[g] = (uint32_t)g;
    uint32_t* dseeds = nullptr;
    if (hipMalloc(&dseeds, sizeof(uint32_t) * G) != hipSuccess) { rvz_destroy(e); *out = nullptr; return RVZ_ENOMEM; }
    int r = hipMemcpy(dseeds, seeds.data(), sizeof(uint32_t) * G, hipMemcpyHostToDevice) == hipSuccess
                ? rvz_env_reset(e, dseeds, nullptr) : RVZ_EHIP;
    if (hipDeviceSynchronize() != hipSuccess) r = RVZ_EHIP;
    (void)hipFree(dseeds);
    if (r != RVZ_OK) { g_create_error = e->err; rvz_destroy(e); *out = nullptr; return r; }
    return RVZ_OK;
}

void rvz_destroy(rvz_engine* e) {
    if (!e) return;
    table_free(e);
    for (hipEvent_t ev : e->ev_pool) (void)hipEventDestroy(ev);
    for (void* p : e->allocs)
        if (p) (void)hipFree(p);
    delete e;
}

int rvz_set_stream(rvz_engine* e, void* stream) {
    if (!e) return RVZ_EINVAL;
    e->stream = (hipStream_t)stream;
    return RVZ_OK;
}

int rvz_sync(rvz_engine* e) {
    if (!e) return RVZ_EINVAL;
    RVZ_HIP(hipStreamSynchronize(e->stream), e);
    return RVZ_OK;
}

int rvz_check(rvz_engine* e, int32_t* host_err) {
    if (!e) return RVZ_EINVAL;
    int32_t h = 0;
    RVZ_HIP(hipMemcpyAsync(&h, e->v.err, sizeof(int32_t), hipMemcpyDeviceToHost, e->stream), e);
    RVZ_HIP(hipStreamSynchronize(e->stream), e);
    if (host_err) *host_err = h;
    if (h) {
        RVZ_HIP(hipMemsetAsync(e->v.err, 0, sizeof(int32_t), e->stream), e);
        e->err = "device error word " + std::to_string(h) +
                 " (1: rng stream exhausted, 2: node pool, 4: path depth, 8: non-finite NN "
                 "value or probability, 16: rvz_play queue wait timed out)";
        return RVZ_EDEVICE;
    }
    return RVZ_OK;
}

#define DISPATCH_BS(e, KERNEL8, KERNEL6) ((e)->BS == 8 ? (KERNEL8) : (KERNEL6))

int rvz_env_reset(rvz_engine* e, const uint32_t* seeds, const uint8_t* mask) {
    if (!e || !seeds) return RVZ_EINVAL;
    e->pending = 0;
    dim3 grid(grid_games(e->v.G)), block(WPB * WAVE);
    if (e->BS == 8) hipLaunchKernelGGL(k_reset<8>, grid, block, 0, e->stream, e->v, seeds, mask);
    else hipLaunchKernelGGL(k_reset<6>, grid, block, 0, e->stream, e->v, seeds, mask);
    e->searching = 0;
    return launch_check(e, "k_reset");
}

int rvz_env_autoreset(rvz_engine* e, const int32_t* idx, int64_t* seeds, int64_t stride,
                      int64_t* plies, int64_t* done, int32_t reset) {
    const Range trace_range("rvz.env.autoreset");
    if (!e || !idx || !plies || (reset && (!seeds || !done))) return RVZ_EINVAL;
    if (reset) e->pending = 0;
    dim3 grid(grid_games(e->v.G)), block(WPB * WAVE);
    if (e->BS == 8) hipLaunchKernelGGL(k_autoreset<8>, grid, block, 0, e->stream, e->v, idx, seeds, stride, plies, done, reset);
    else hipLaunchKernelGGL(k_autoreset<6>, grid, block, 0, e->stream, e->v, idx, seeds, stride, plies, done, reset);
    return launch_check(e, "k_autoreset");
}

int rvz_env_get(rvz_engine* e, uint64_t* black, uint64_t* white, int32_t* status) {
    if (!e) return RVZ_EINVAL;
    const size_t G = e->v.G;
    if (black) RVZ_HIP(hipMemcpyAsync(black, e->v.black, G * 8, hipMemcpyDeviceToDevice, e->stream), e);
    if (white) RVZ_HIP(hipMemcpyAsync(white, e->v.white, G * 8, hipMemcpyDeviceToDevice, e->stream), e);
    if (status) RVZ_HIP(hipMemcpyAsync(status, e->v.status, G * 16, hipMemcpyDeviceToDevice, e->stream), e);
    return RVZ_OK;
}

// The memo's carried links hold only while each search follows the previous one's move
// (rvz_act with apply): a position set or moved from the host, or an abandoned search, drops them.
static int memo_drop(rvz_engine* e) {
    if (!e->v.memo) return RVZ_OK;
    RVZ_HIP(fill32_async(e->v.carry, LINK_NONE, (size_t)e->v.G, e->stream), e);
    return RVZ_OK;
}

int rvz_env_set(rvz_engine* e, const uint64_t* black, const uint64_t* white, const int32_t* status) {
    if (!e || !black || !white || !status) return RVZ_EINVAL;
    e->pending = 0;
    if (memo_drop(e) != RVZ_OK) return RVZ_EHIP;
    const size_t G = e->v.G;
    RVZ_HIP(hipMemcpyAsync(e->v.black, black, G * 8, hipMemcpyDeviceToDevice, e->stream), e);
    RVZ_HIP(hipMemcpyAsync(e->v.white, white, G * 8, hipMemcpyDeviceToDevice, e->stream), e);
    RVZ_HIP(hipMemcpyAsync(e->v.status, status, G * 16, hipMemcpyDeviceToDevice, e->stream), e);
    e->searching = 0;
    return RVZ_OK;
}

int rvz_env_set_draws(rvz_engine* e, const double* u) {
    static_assert(RNG_DRAWS == RVZ_DRAWS, "include/rvz.h's RVZ_DRAWS is the stream length");
    if (!e || !u) return RVZ_EINVAL;
    const size_t G = e->v.G;
    RVZ_HIP(hipMemcpyAsync(e->v.rng_u, u, G * RNG_DRAWS * sizeof(double), hipMemcpyDeviceToDevice,
                           e->stream), e);
    RVZ_HIP(hipMemsetAsync(e->v.rng_pos, 0, G * sizeof(int32_t), e->stream), e);
    return RVZ_OK;
}

int rvz_env_draws(rvz_engine* e, int32_t* out_pos) {
    if (!e || !out_pos) return RVZ_EINVAL;
    RVZ_HIP(hipMemcpyAsync(out_pos, e->v.rng_pos, (size_t)e->v.G * sizeof(int32_t),
                           hipMemcpyDeviceToDevice, e->stream), e);
    return RVZ_OK;
}

int rvz_board_legal(int32_t bs, int32_t n, const uint64_t* black, const uint64_t* white,
                    const int32_t* status, uint64_t* out, void* stream) {
    if ((bs != 8 && bs != 6) || n < 0 || (n > 0 && (!black || !white || !status || !out)))
        return RVZ_EINVAL;
    if (n == 0) return RVZ_OK;
    dim3 grid((n + 255) / 256), block(256);
    if (bs == 8) hipLaunchKernelGGL(k_board_legal<8>, grid, block, 0, (hipStream_t)stream, n, black, white, status, out);
    else hipLaunchKernelGGL(k_board_legal<6>, grid, block, 0, (hipStream_t)stream, n, black, white, status, out);
    return hipGetLastError() == hipSuccess ? RVZ_OK : RVZ_EHIP;
}

int rvz_board_apply(int32_t bs, int32_t n, uint64_t* black, uint64_t* white, int32_t* status,
                    const int32_t* sq, int32_t* ok, void* stream) {
    if ((bs != 8 && bs != 6) || n < 0 || (n > 0 && (!black || !white || !status || !sq)))
        return RVZ_EINVAL;
    if (n == 0) return RVZ_OK;
    dim3 grid((n + 255) / 256), block(256);
    if (bs == 8) hipLaunchKernelGGL(k_board_apply<8>, grid, block, 0, (hipStream_t)stream, n, black, white, status, sq, ok);
    else hipLaunchKernelGGL(k_board_apply<6>, grid, block, 0, (hipStream_t)stream, n, black, white, status, sq, ok);
    return hipGetLastError() == hipSuccess ? RVZ_OK : RVZ_EHIP;
}

int rvz_board_canonical(int32_t bs, int32_t n, const uint64_t* black, const uint64_t* white,
                        const int32_t* status, float* out, void* stream) {
    if ((bs != 8 && bs != 6) || n < 0 || (n > 0 && (!black || !white || !status || !out)))
        return RVZ_EINVAL;
    if (n == 0) return RVZ_OK;
    const int total = n * bs * bs;
    dim3 grid((total + 255) / 256), block(256);
    if (bs == 8) hipLaunchKernelGGL(k_board_canonical<8>, grid, block, 0, (hipStream_t)stream, n, black, white, status, out);
    else hipLaunchKernelGGL(k_board_canonical<6>, grid, block, 0, (hipStream_t)stream, n, black, white, status, out);
    return hipGetLastError() == hipSuccess ? RVZ_OK : RVZ_EHIP;
}

int rvz_policy_softmax(int32_t bs, int32_t n, const float* logits, float* probs, void* stream) {
    if ((bs != 8 && bs != 6) || n < 0 || (n > 0 && (!logits || !probs))) return RVZ_EINVAL;
    if (n == 0) return RVZ_OK;
    dim3 grid((n + WPB - 1) / WPB), block(WPB * WAVE);
    if (bs == 8) hipLaunchKernelGGL(k_policy_softmax<8>, grid, block, 0, (hipStream_t)stream, n, logits, probs);
    else hipLaunchKernelGGL(k_policy_softmax<6>, grid, block, 0, (hipStream_t)stream, n, logits, probs);
    return hipGetLastError() == hipSuccess ? RVZ_OK : RVZ_EHIP;
}

int rvz_env_legal(rvz_engine* e, uint64_t* out) {
    if (!e) return RVZ_EINVAL;
    int r = rvz_board_legal(e->BS, e->v.G, e->v.black, e->v.white, e->v.status, out, e->stream);
    if (r != RVZ_OK) e->err = "rvz_env_legal launch failed";
    else e->counters[1] += 1;
    return r;
}

int rvz_env_apply(rvz_engine* e, const int32_t* sq, int32_t* ok) {
    const Range trace_range("rvz.env.apply");
    if (!e) return RVZ_EINVAL;
    if (memo_drop(e) != RVZ_OK) return RVZ_EHIP;
    int r = rvz_board_apply(e->BS, e->v.G, e->v.black, e->v.white, e->v.status, sq, ok, e->stream);
    if (r != RVZ_OK) e->err = "rvz_env_apply launch failed";
    else e->counters[1] += 1;
    e->searching = 0;
    return r;
}

int rvz_search_begin(rvz_engine* e) {
    const Range trace_range("rvz.search.begin");
    if (!e) return RVZ_EINVAL;
    if (e->searching && e->next_batch > 0 && memo_drop(e) != RVZ_OK) return RVZ_EHIP;
    e->next_batch = 0;
    e->searching = 1;
    if (e->v.live && e->live_dirty) {   // an abandoned search left counts behind
        RVZ_HIP(fill32_async(e->v.live, 0u, (size_t)e->E * e->v.NS * RVZ_LIVE_PITCH, e->stream),
                e);
        e->live_dirty = 0;
    }
    e->pending = 0;  // an unconsumed submit of an abandoned search is dropped
    return RVZ_OK;
}

int rvz_search_step(rvz_engine* e, void* leaf_x, int32_t* need) {
    const Range trace_range("rvz.search.step (expand/backup + select)");
    if (!e || !leaf_x || !need) return RVZ_EINVAL;
    if (!e->searching) { e->err = "rvz_search_step before rvz_search_begin"; return RVZ_EINVAL; }
    const int S = e->cfg.num_simulations, B = e->cfg.batch_size;
    const int start = e->next_batch * B;
    if (start >= S) return RVZ_DONE;
    const int bsz = S - start < B ? S - start : B;
    const int first = e->next_batch == 0;
    const int ex = e->pending;
    const float* pol = e->pend_policy;
    const float* val = e->pend_value;
    const int lg = e->pend_is_logits;
    dim3 grid(grid_games(e->v.G)), block(WPB * WAVE);
    timing_begin(e, 0);
    if (e->cfg.leaf_dtype == RVZ_LEAF_F32) {
        float* x = (float*)leaf_x;
        if (e->BS == 8) hipLaunchKernelGGL((k_step<8, float>), grid, block, 0, e->stream, e->v, ex, pol, lg, val, first, bsz, e->next_batch, x, need);
        else hipLaunchKernelGGL((k_step<6, float>), grid, block, 0, e->stream, e->v, ex, pol, lg, val, first, bsz, e->next_batch, x, need);
    } else {
        __hip_bfloat16* x = (__hip_bfloat16*)leaf_x;
        if (e->BS == 8) hipLaunchKernelGGL((k_step<8, __hip_bfloat16>), grid, block, 0, e->stream, e->v, ex, pol, lg, val, first, bsz, e->next_batch, x, need);
        else hipLaunchKernelGGL((k_step<6, __hip_bfloat16>), grid, block, 0, e->stream, e->v, ex, pol, lg, val, first, bsz, e->next_batch, x, need);
    }
    timing_end(e);
    e->pending = 0;
    e->next_batch += 1;
    if (e->v.live) e->live_dirty = 1;
    e->counters[0] += 1;
    return launch_check(e, "k_step");
}

int rvz_search_submit(rvz_engine* e, const float* policy, int32_t is_logits, const float* value) {
    const Range trace_range("rvz.search.submit");
    if (!e || !policy || !value) return RVZ_EINVAL;
    if (!e->searching || e->next_batch == 0) {
        e->err = "rvz_search_submit without a preceding rvz_search_step";
        return RVZ_EINVAL;
    }
    if (e->pending) { e->err = "rvz_search_submit twice for one batch"; return RVZ_EINVAL; }
    // deferred: the expand + backup runs at the head of the next k_step / k_act launch (or of
    // k_expand_backup for rvz_search_visits); policy/value must stay valid until then.
    e->pending = 1;
    e->pend_policy = policy;
    e->pend_value = value;
    e->pend_is_logits = is_logits;
    return RVZ_OK;
}

static int flush_pending(rvz_engine* e) {
    if (!e->pending) return RVZ_OK;
    dim3 grid(grid_games(e->v.G)), block(WPB * WAVE);
    if (e->BS == 8) hipLaunchKernelGGL(k_expand_backup<8>, grid, block, 0, e->stream, e->v, e->pending, e->pend_policy, e->pend_is_logits, e->pend_value);
    else hipLaunchKernelGGL(k_expand_backup<6>, grid, block, 0, e->stream, e->v, e->pending, e->pend_policy, e->pend_is_logits, e->pend_value);
    e->pending = 0;
    return launch_check(e, "k_expand_backup");
}

int rvz_search_visits(rvz_engine* e, int32_t* out) {
    if (!e || !out) return RVZ_EINVAL;
    int r = flush_pending(e);
    if (r != RVZ_OK) return r;
    dim3 grid(grid_games(e->v.G)), block(WPB * WAVE);
    if (e->BS == 8) hipLaunchKernelGGL(k_visits<8>, grid, block, 0, e->stream, e->v, out);
    else hipLaunchKernelGGL(k_visits<6>, grid, block, 0, e->stream, e->v, out);
    return launch_check(e, "k_visits");
}

int rvz_search_compact(rvz_engine* e, int32_t on) {
    if (!e) return RVZ_EINVAL;
    if (e->pending || (e->searching && e->next_batch > 0)) {
        e->err = "rvz_search_compact inside a search";
        return RVZ_EINVAL;
    }
    if (on && !e->live_buf) {
        // [E] live counts, [G] row map, then the 8-byte running total
        const size_t nlive = (size_t)e->E * e->v.NS * RVZ_LIVE_PITCH;
        const size_t words = (nlive + e->v.G + 1) / 2 * 2 + 2;
        e->live_buf = dalloc<int32_t>(e, words);
        if (!e->live_buf) { e->err = "hipMalloc failed (live counts)"; return RVZ_ENOMEM; }
        RVZ_HIP(hipMemsetAsync(e->live_buf, 0, sizeof(int32_t) * words, e->stream), e);
        e->live_total = reinterpret_cast<unsigned long long*>(e->live_buf + words - 2);
        e->live_dirty = 0;
    }
    e->v.live = on ? e->live_buf : nullptr;
    e->v.row_of = on ? e->live_buf + (size_t)e->E * e->v.NS * RVZ_LIVE_PITCH : nullptr;
    e->v.live_total = on ? e->live_total : nullptr;
    return RVZ_OK;
}

// The memo needs the node pool's second half (the previous search's tree stays readable while a
// search writes the other half): the first rvz_search_memo(on) reallocates nodes and meta with
// M = 1 + 2 E S^2. Outside a search no tree is live (the carried links are dropped here anyway),
// so nothing is copied. Pointers held by an already captured graph would dangle: enable the memo
// before capturing (rvz.Engine does it in its constructor).
static int memo_grow(rvz_engine* e) {
    const int M2 = 1 + 2 * e->E * e->NSQ;
    if (e->M == M2) return RVZ_OK;
    const size_t G = e->v.G;
    Node* nodes = nullptr;
    uint32_t* meta = nullptr;
    if (hipMalloc(reinterpret_cast<void**>(&nodes), G * M2 * sizeof(Node)) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&meta), G * M2 * sizeof(uint32_t)) != hipSuccess) {
        if (nodes) (void)hipFree(nodes);
        e->err = "hipMalloc failed (the memo's second node-pool half)";
        return RVZ_ENOMEM;
    }
    RVZ_HIP(hipStreamSynchronize(e->stream), e);   // no launch may still read the old pool
    for (void*& p : e->allocs) {
        if (p == e->v.nodes) { (void)hipFree(p); p = nodes; }
        else if (p == e->v.meta) { (void)hipFree(p); p = meta; }
    }
    e->v.nodes = nodes;
    e->v.meta = meta;
    e->M = e->v.M = M2;
    RVZ_HIP(hipMemsetAsync(meta, 0, G * M2 * sizeof(uint32_t), e->stream), e);
    return RVZ_OK;
}

int rvz_search_memo(rvz_engine* e, int32_t on) {
    if (!e) return RVZ_EINVAL;
    if (e->pending || (e->searching && e->next_batch > 0)) {
        e->err = "rvz_search_memo inside a search";
        return RVZ_EINVAL;
    }
    if (on) {
        const int r = memo_grow(e);
        if (r != RVZ_OK) return r;
    }
    e->v.memo = 1;             // so that memo_drop clears the links either way
    if (memo_drop(e) != RVZ_OK) return RVZ_EHIP;
    e->v.memo = on ? 1 : 0;
    return RVZ_OK;
}

int rvz_search_memo_reset(rvz_engine* e) {
    if (!e) return RVZ_EINVAL;
    const int r = memo_drop(e);
    return r != RVZ_OK ? r : table_bump(e);   // new weights: the table's rows are stale too
}

int rvz_play_gate(rvz_engine* e, double fraction, double timeout_us, double late_us) {
    if (!e || !(fraction <= 1.0) || !(timeout_us >= 0.0) || !(late_us >= 0.0) ||
        timeout_us > 1e6 || late_us > 1e6) {
        if (e) e->err = "rvz_play_gate: fraction <= 1 (< 0: the default), 0 <= us <= 1e6";
        return RVZ_EINVAL;
    }
    e->gate_frac = fraction;
    e->gate_us = timeout_us;
    e->gate_late_us = late_us;
    return RVZ_OK;
}

int rvz_play_table(rvz_engine* e, int64_t slots, int32_t max_discs) {
    if (!e) return RVZ_EINVAL;
    if (slots != 0 && (slots < 1024 || (slots & (slots - 1)) != 0 || slots > (1ll << 30) ||
                       max_discs < 4)) {
        e->err = "rvz_play_table: slots a power of two in [1024, 2^30] (or 0), max_discs >= 4";
        return RVZ_EINVAL;
    }
    RVZ_HIP(hipStreamSynchronize(e->stream), e);
    if (slots == e->tslots && slots != 0) {   // same size: new limit, a fresh generation
        e->tmaxd = max_discs;
        return table_bump(e);
    }
    table_free(e);
    if (slots == 0) return RVZ_OK;
    const size_t stride = e->BS == 8 ? TabGeo<8>::STRIDE : TabGeo<6>::STRIDE;
    if (hipMalloc(reinterpret_cast<void**>(&e->tab), (size_t)slots * stride * 8) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&e->tclaim), (size_t)slots * 4) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&e->tgen), 4) != hipSuccess) {
        table_free(e);
        e->err = "hipMalloc failed (rvz_play_table)";
        return RVZ_ENOMEM;
    }
    hipError_t st = hipMemset(e->tab, 0, (size_t)slots * stride * 8);   // tags 0: no generation
    if (st == hipSuccess) st = hipMemset(e->tclaim, 0, (size_t)slots * 4);
    if (st == hipSuccess) st = hipMemsetD32(e->tgen, 1u, 1);
    if (st == hipSuccess) st = hipDeviceSynchronize();
    if (st != hipSuccess) {
        table_free(e);
        e->err = std::string("rvz_play_table init: ") + hipGetErrorString(st);
        return RVZ_EHIP;
    }
    e->tslots = slots;
    e->tmaxd = max_discs;
    return RVZ_OK;
}

int rvz_search_rows_total(rvz_engine* e, int64_t* out) {
    if (!e || !out) return RVZ_EINVAL;
    *out = 0;
    if (!e->live_total) return RVZ_OK;
    unsigned long long h = 0;
    RVZ_HIP(hipMemcpyAsync(&h, e->live_total, sizeof(h), hipMemcpyDeviceToHost, e->stream), e);
    RVZ_HIP(hipStreamSynchronize(e->stream), e);
    *out = (int64_t)h;
    return RVZ_OK;
}

const int32_t* rvz_search_live_count(const rvz_engine* e) {
    if (!e || !e->v.live || e->next_batch == 0) return nullptr;
    return e->v.live + (size_t)(e->next_batch - 1) * e->v.NS * RVZ_LIVE_PITCH;
}

#ifdef RVZ_WALK_STATS
// host int64[10]: sums over games of the 5 walk counters, then their maxima; zeroes them
int rvz_walk_stats(int32_t n_games, int64_t* out10) {
    static std::vector<unsigned int> h;
    const int n = n_games < WALK_STATS_MAX ? n_games : WALK_STATS_MAX;
    h.assign((size_t)n * 5, 0u);
    if (hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(g_walk), h.size() * 4) != hipSuccess)
        return RVZ_EHIP;
    for (int i = 0; i < 10; ++i) out10[i] = 0;
    for (int gi = 0; gi < n; ++gi)
        for (int i = 0; i < 5; ++i) {
            out10[i] += h[(size_t)gi * 5 + i];
            if ((int64_t)h[(size_t)gi * 5 + i] > out10[5 + i]) out10[5 + i] = h[(size_t)gi * 5 + i];
        }
    std::vector<unsigned int> z((size_t)WALK_STATS_MAX * 5, 0u);
    return hipMemcpyToSymbol(HIP_SYMBOL(g_walk), z.data(), z.size() * 4) == hipSuccess
               ? RVZ_OK : RVZ_EHIP;
}

// host int64[11]: the 5 shader-clock categories of the game with the largest total, then the
// means over games, then that game's index; zeroes them
int rvz_walk_times(int32_t n_games, int64_t* out11) {
    static std::vector<unsigned long long> h;
    const int n = n_games < WALK_STATS_MAX ? n_games : WALK_STATS_MAX;
    h.assign((size_t)n * 5, 0ull);
    if (hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(g_wtime), h.size() * 8) != hipSuccess)
        return RVZ_EHIP;
    int best = 0;
    unsigned long long bt = 0;
    double mean[5] = {0, 0, 0, 0, 0};
    for (int gi = 0; gi < n; ++gi) {
        unsigned long long t = 0;
        for (int i = 0; i < 5; ++i) {
            t += h[(size_t)gi * 5 + i];
            mean[i] += (double)h[(size_t)gi * 5 + i] / n;
        }
        if (t > bt) { bt = t; best = gi; }
    }
    for (int i = 0; i < 5; ++i) {
        out11[i] = (int64_t)h[(size_t)best * 5 + i];
        out11[5 + i] = (int64_t)mean[i];
    }
    out11[10] = best;
    std::vector<unsigned long long> z((size_t)WALK_STATS_MAX * 5, 0ull);
    return hipMemcpyToSymbol(HIP_SYMBOL(g_wtime), z.data(), z.size() * 8) == hipSuccess
               ? RVZ_OK : RVZ_EHIP;
}
#endif

#ifdef RVZ_WALK_STATS
// tools/exp_play_walks.py: host uint64 [n][9] = g_wtime's 5 columns, then g_ftime's 4; zeroes both
int rvz_play_walk_read(int32_t n_games, uint64_t* out) {
    const int n = n_games < WALK_STATS_MAX ? n_games : WALK_STATS_MAX;
    std::vector<unsigned long long> a((size_t)n * 5), b((size_t)n * 4);
    if (hipMemcpyFromSymbol(a.data(), HIP_SYMBOL(g_wtime), a.size() * 8) != hipSuccess ||
        hipMemcpyFromSymbol(b.data(), HIP_SYMBOL(g_ftime), b.size() * 8) != hipSuccess)
        return RVZ_EHIP;
    for (int i = 0; i < n; ++i) {
        for (int k = 0; k < 5; ++k) out[(size_t)i * 9 + k] = a[(size_t)i * 5 + k];
        for (int k = 0; k < 4; ++k) out[(size_t)i * 9 + 5 + k] = b[(size_t)i * 4 + k];
    }
    std::vector<unsigned long long> z((size_t)WALK_STATS_MAX * 5, 0ull);
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_wtime), z.data(), z.size() * 8) != hipSuccess)
        return RVZ_EHIP;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_ftime), z.data(), (size_t)WALK_STATS_MAX * 4 * 8) ==
                   hipSuccess ? RVZ_OK : RVZ_EHIP;
}
#endif

int rvz_search_skip(rvz_engine* e) {
    if (!e) return RVZ_EINVAL;
    const int S = e->cfg.num_simulations, B = e->cfg.batch_size;
    if (!e->searching || e->next_batch == 0 || e->next_batch * B < S) {
        e->err = "rvz_search_skip is only valid after the last rvz_search_step of a search";
        return RVZ_EINVAL;
    }
    if (e->pending) { e->err = "rvz_search_skip after rvz_search_submit"; return RVZ_EINVAL; }
    if (S <= B) {     // one batch: its leaf is the root, whose expansion the act needs
        e->err = "rvz_search_skip needs a search of at least two batches (num_simulations > "
                 "batch_size): a single batch's leaf is the root";
        return RVZ_EINVAL;
    }
    e->pending = 2;   // rvz_act: visit counts only
    return RVZ_OK;
}

int rvz_act(rvz_engine* e, double temperature, const double* u, int32_t apply, int32_t* out_idx,
            double* out_p) {
    const Range trace_range("rvz.act (expand/backup + action + move)");
    if (!e || !out_idx || !out_p) return RVZ_EINVAL;
    const int ex = e->pending;
    dim3 grid(grid_games(e->v.G)), block(WPB * WAVE);
    timing_begin(e, 1);
    if (e->BS == 8) hipLaunchKernelGGL(k_act<8>, grid, block, 0, e->stream, e->v, ex, e->pend_policy, e->pend_is_logits, e->pend_value, temperature, u, apply, out_idx, out_p);
    else hipLaunchKernelGGL(k_act<6>, grid, block, 0, e->stream, e->v, ex, e->pend_policy, e->pend_is_logits, e->pend_value, temperature, u, apply, out_idx, out_p);
    timing_end(e);
    e->pending = 0;
    e->live_dirty = 0;
    if (apply) e->searching = 0;
    return launch_check(e, "k_act");
}

static int64_t play_al4(int64_t n) { return (n + 3) / 4 * 4; }

// scratch (floats): [queue words: q_next + pad, q_done[G]] (one 16-B-aligned block at the start,
// zeroed per launch), leaf planes, need, head-conv rows, logits, value
// + the pass gate's words (PlayArgs::gate: 8 XCDs x 128 bytes)
static int64_t play_qwords(int64_t G) { return 4 + play_al4(G) + 8 * 32; }
int64_t rvz_play_scratch_size(const rvz_engine* e) {
    if (!e) return RVZ_EINVAL;
    const int64_t G = e->v.G;
    return play_qwords(G) + play_al4(G * 3 * e->NSQ) + play_al4(G) + play_al4(G * 192) +
           play_al4(G * e->NPOL) + play_al4(G);
}

#ifndef RVZ_PLAY_GROUP
#define RVZ_PLAY_GROUP 4      // games per task of the queue schedule
#endif
// the pass gate's default (rvz_play_gate; measured on C3, profiles/r06c_gate_ab_*): a round opens
// when 0.8 of the XCD's running workgroups arrived or 400 us after a waiter's arrival; a workgroup
// arriving within 200 us of a round's opening joins it at once
#ifndef RVZ_PLAY_GATE_FRAC
#define RVZ_PLAY_GATE_FRAC 0.8
#endif
#ifndef RVZ_PLAY_GATE_US
#define RVZ_PLAY_GATE_US 400.0
#endif
#ifndef RVZ_PLAY_GATE_LATE_US
#define RVZ_PLAY_GATE_LATE_US 200.0
#endif
extern "C++" {
template <int F, int NB, int CTW, int PTW, int BS, int OCC>
static int play_launch(rvz_engine* e, const View& v, const PlayArgs& pa, int slots_per_cu) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, e->cfg.device) !=
            hipSuccess || cus <= 0)
        cus = 256;
    PlayArgs a = pa;
    const int slots = cus * slots_per_cu;
    dim3 grid;
    if (a.q_next) {     // queue: one persistent workgroup per resident slot, groups of gpw games
        if (a.gpw <= 0) a.gpw = RVZ_PLAY_GROUP;
        if (a.gpw > play_gpw_max<F, BS>()) a.gpw = play_gpw_max<F, BS>();
        a.n_groups = (v.G + a.gpw - 1) / a.gpw;
        grid = dim3(a.n_groups < slots ? a.n_groups : slots);
        RVZ_HIP(fill32_async(a.q_next, 0u, (size_t)play_qwords(v.G), e->stream), e);
    } else {            // static: workgroup w owns group w for every ply
        if (a.gpw <= 0) a.gpw = (v.G + slots - 1) / slots;
        if (a.gpw > play_gpw_max<F, BS>()) a.gpw = play_gpw_max<F, BS>();
        a.n_groups = (v.G + a.gpw - 1) / a.gpw;
        grid = dim3(a.n_groups);
    }
    PlayCtx ctx;
    ctx.v = v;
    ctx.a = a;
    hipLaunchKernelGGL((k_play<F, NB, CTW, PTW, BS, OCC>), grid, dim3(256), 0, e->stream, ctx);
    return launch_check(e, "k_play");
}
}  // extern "C++"

#ifdef RVZ_PLAY_TIMING
// tools/exp_play_phases.py: host copy of g_play_t (n workgroups x 12) and g_pass_t (n x 6), then
// zeroed
int rvz_play_timing_read(uint64_t* host, int n) {
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_play_t), (size_t)n * 12 * 8) != hipSuccess)
        return RVZ_EHIP;
    if (hipMemcpyFromSymbol(host + (size_t)n * 12, HIP_SYMBOL(g_pass_t), (size_t)n * 6 * 8) !=
        hipSuccess)
        return RVZ_EHIP;
    std::vector<unsigned long long> z((size_t)16384 * 12, 0ull);
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_pass_t), z.data(), (size_t)16384 * 6 * 8) != hipSuccess)
        return RVZ_EHIP;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_play_t), z.data(), z.size() * 8) == hipSuccess
               ? RVZ_OK : RVZ_EHIP;
}
#endif


int rvz_play(rvz_engine* e, const rvz_play_args* a) {
    const Range trace_range("rvz.play (fused search + h2 evaluator)");
    if (!e || !a) return RVZ_EINVAL;
    if (!a->params || !a->blob || !a->scratch || !a->seeds || !a->plies_done || !a->out_idx ||
        !a->out_p || (a->reset && !a->games_done) || a->plies < 1 || a->blocks < 0 ||
        (a->filters != 64 && a->filters != 128 && !(a->filters == 256 && e->BS == 8)) ||
        a->games_per_workgroup < -PLAY_GPW_MAX ||
        e->cfg.leaf_dtype != RVZ_LEAF_F32) {
        e->err = "rvz_play: invalid arguments";
        return RVZ_EINVAL;
    }
    if ((((uintptr_t)a->params | (uintptr_t)a->blob | (uintptr_t)a->scratch) & 15) != 0) {
        e->err = "rvz_play: params, blob and scratch must be 16-byte aligned";
        return RVZ_EINVAL;
    }
    if (e->pending || (e->searching && e->next_batch > 0)) {
        e->err = "rvz_play inside a search";
        return RVZ_EINVAL;
    }
    View v = e->v;
    v.live = nullptr;       // the workgroups compact their own rows
    v.row_of = nullptr;
    v.live_total = nullptr;
    v.stats = nullptr;
    const int64_t G = v.G;
    PlayArgs pa;
    pa.prm = a->params;
    pa.L = make_layout(a->filters, a->blocks, e->BS);
    pa.blob = a->blob;
    pa.n_blocks = a->blocks;
    float* sc = a->scratch;
    // games_per_workgroup > 0: static groups of that size; <= 0: the task queue, groups of
    // -games_per_workgroup games (0: RVZ_PLAY_GROUP)
    const bool queue = a->games_per_workgroup <= 0;
    pa.q_next = queue ? reinterpret_cast<unsigned*>(sc) : nullptr;
    pa.q_done = queue ? reinterpret_cast<unsigned*>(sc) + 4 : nullptr;
    pa.n_groups = 0;
    // the per-XCD pass gate (rvz_play.hip.h play_gate, rvz_play_gate; 8x8 at 128 / 256 filters, queue
    // schedule only: its words are zeroed with the queue's)
    pa.gate = queue ? reinterpret_cast<unsigned long long*>(sc + 4 + play_al4(G)) : nullptr;
    {   // rvz_play_gate's setting (default: RVZ_PLAY_GATE_DEFAULT), RVZ_PLAY_GATE overriding it
        double frac = e->gate_frac, us = e->gate_us, late = e->gate_late_us;
        if (frac < 0.0) {
            frac = RVZ_PLAY_GATE_FRAC;
            us = RVZ_PLAY_GATE_US;
            late = RVZ_PLAY_GATE_LATE_US;
        }
        if (const char* gs = getenv("RVZ_PLAY_GATE")) {   // "fraction,us[,late_us]" or "off"
            double f = 0.0, u = 0.0, l = 0.0;
            const int n = sscanf(gs, "%lf,%lf,%lf", &f, &u, &l);
            frac = n >= 2 ? f : 0.0;
            us = u;
            late = n >= 3 ? l : 0.0;
        }
        pa.gate_frac = (queue && frac > 0.0 && us > 0.0)
                           ? (unsigned)(fmin(frac, 1.0) * 65536.0 + 0.5) : 0u;
        pa.gate_t = (unsigned)(us * 100.0);
        pa.gate_late = late > 0.0 ? (unsigned)(late * 100.0) : 0u;
    }
    sc += play_qwords(G);
    pa.x = sc;
    sc += play_al4(G * 3 * e->NSQ);
    pa.need = reinterpret_cast<int32_t*>(sc);
    sc += play_al4(G);
    pa.work = sc;
    sc += play_al4(G * 192);
    pa.logits = sc;
    sc += play_al4(G * e->NPOL);
    pa.value = sc;
    pa.ovf = a->ovf;
    pa.gpw = queue ? -a->games_per_workgroup : a->games_per_workgroup;
    pa.plies = a->plies;
    // a search of one batch (S <= B) evaluates it: its leaf is the root, which the act needs
    // expanded (the deferred last batch is dead only from the second batch on)
    pa.skip_last = a->skip_last_eval && e->cfg.num_simulations > e->cfg.batch_size ? 1 : 0;
    pa.reset = a->reset ? 1 : 0;
    pa.S = e->cfg.num_simulations;
    pa.B = e->cfg.batch_size;
    pa.temperature = a->temperature;
    pa.seeds = a->seeds;
    pa.stride = a->seed_stride;
    pa.ply_ctr = a->plies_done;
    pa.done = a->games_done;
    pa.out_idx = a->out_idx;
    pa.out_p = a->out_p;
    pa.hist = a->hist;
    pa.rows = reinterpret_cast<unsigned long long*>(a->rows_evaluated);
    pa.budget = a->ply_budget;
    pa.tab = nullptr;
    pa.tclaim = nullptr;
    pa.tgen = nullptr;
    pa.tmask = 0;
    pa.tmaxd = 0;
    pa.tstats = reinterpret_cast<unsigned long long*>(a->table_stats);
    pa.rec_black = a->rec_black;
    pa.rec_white = a->rec_white;
    pa.rec_side = a->rec_side;
    pa.rec_p = a->rec_p;
    if ((a->rec_black || a->rec_white || a->rec_side || a->rec_p) &&
        !(a->rec_black && a->rec_white && a->rec_side && a->rec_p)) {
        e->err = "rvz_play: rec_black, rec_white, rec_side and rec_p go together";
        return RVZ_EINVAL;
    }
    if (e->tab) {
        if (e->tab_blob != a->blob) {   // other weights than the generation's rows came from
            if (e->tab_blob) {
                // the generation bump is a kernel on the stream: inside a capture it would be
                // recorded and replayed, invalidating the table on every replay
                hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
                if (hipStreamIsCapturing(e->stream, &cs) == hipSuccess &&
                    cs != hipStreamCaptureStatusNone) {
                    e->err = "rvz_play: another weight blob than the table's while the stream is "
                             "capturing (play once eagerly with this evaluator before capturing)";
                    return RVZ_EINVAL;
                }
                const int r = table_bump(e);
                if (r != RVZ_OK) return r;
            }
            e->tab_blob = a->blob;
        }
        pa.tab = e->tab;
        pa.tclaim = e->tclaim;
        pa.tgen = e->tgen;
        pa.tmask = (unsigned)(e->tslots - 1);
        pa.tmaxd = e->tmaxd;
    }
    // the queue's bounded wait (device error 16 when exceeded); RVZ_PLAY_SPIN_LIMIT lowers it to
    // inject the timeout in tests (tests/test_gpu_play.py)
    pa.spin_limit = 1u << 26;
    if (const char* sl = getenv("RVZ_PLAY_SPIN_LIMIT")) pa.spin_limit = (unsigned)strtoul(sl, nullptr, 10);
    e->searching = 0;
    if (e->BS == 8)
        return a->filters == 64    ? play_launch<64, 2, 2, 4, 8, 2>(e, v, pa, 2)
               : a->filters == 128 ? play_launch<128, 1, 2, 4, 8, 2>(e, v, pa, 2)
                                   : play_launch<256, 1, 4, 4, 8, 1>(e, v, pa, 1);
    return a->filters == 64 ? play_launch<64, 3, 2, 4, 6, 2>(e, v, pa, 2)
                            : play_launch<128, 1, 2, 3, 6, 2>(e, v, pa, 2);
}

// ---- stream-ordered HIP event timer without system fence (bench.py: per-launch kernel
// durations in eager plies; torch's events carry a system-scope fence that adds tens of us)
struct rvz_timer {
    std::vector<hipEvent_t> ev;
};

int rvz_timer_create(int32_t n, rvz_timer** out) {
    if (n <= 0 || !out) return RVZ_EINVAL;
    rvz_timer* t = new rvz_timer;
    t->ev.resize(n, nullptr);
    for (auto& e : t->ev) {
        if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) {
            for (auto& f : t->ev)
                if (f) (void)hipEventDestroy(f);
            delete t;
            return RVZ_EHIP;
        }
    }
    *out = t;
    return RVZ_OK;
}

int rvz_timer_record(rvz_timer* t, int32_t i, void* stream) {
    if (!t || i < 0 || i >= (int32_t)t->ev.size()) return RVZ_EINVAL;
    return hipEventRecord(t->ev[i], (hipStream_t)stream) == hipSuccess ? RVZ_OK : RVZ_EHIP;
}

int rvz_timer_elapsed(rvz_timer* t, int32_t i, int32_t j, float* ms) {
    if (!t || !ms || i < 0 || j < 0 || i >= (int32_t)t->ev.size() || j >= (int32_t)t->ev.size())
        return RVZ_EINVAL;
    if (hipEventSynchronize(t->ev[j]) != hipSuccess) return RVZ_EHIP;
    return hipEventElapsedTime(ms, t->ev[i], t->ev[j]) == hipSuccess ? RVZ_OK : RVZ_EHIP;
}

void rvz_timer_destroy(rvz_timer* t) {
    if (!t) return;
    for (auto& e : t->ev)
        if (e) (void)hipEventDestroy(e);
    delete t;
}

int rvz_counters(const rvz_engine* e, int64_t* out2) {
    if (!e || !out2) return RVZ_EINVAL;
    out2[0] = e->counters[0];
    out2[1] = e->counters[1];
    return RVZ_OK;
}

int rvz_stats_enable(rvz_engine* e, int32_t on) {
    if (!e) return RVZ_EINVAL;
    e->v.stats = on ? e->stats_buf : nullptr;
    if (on) RVZ_HIP(hipMemsetAsync(e->stats_buf, 0, 3 * (size_t)e->v.G * sizeof(unsigned long long), e->stream), e);
    return RVZ_OK;
}

int rvz_stats_read(rvz_engine* e, int64_t* out3) {
    if (!e || !out3) return RVZ_EINVAL;
    const size_t G = e->v.G;
    std::vector<unsigned long long> h(3 * G);
    RVZ_HIP(hipMemcpyAsync(h.data(), e->stats_buf, h.size() * sizeof(unsigned long long),
                           hipMemcpyDeviceToHost, e->stream), e);
    RVZ_HIP(hipStreamSynchronize(e->stream), e);
    for (int k = 0; k < 3; ++k) {
        unsigned long long t = 0;
        for (size_t g = 0; g < G; ++g) t += h[k * G + g];
        out3[k] = (int64_t)t;
    }
    return RVZ_OK;
}

int rvz_timing_enable(rvz_engine* e, int32_t on) {
    if (!e) return RVZ_EINVAL;
    e->timing = on ? 1 : 0;
    e->ev_used = 0;
    e->ev_marks.clear();
    return RVZ_OK;
}

int rvz_timing_read(rvz_engine* e, double* out_ms, int32_t* out_n) {
    if (!e || !out_ms || !out_n) return RVZ_EINVAL;
    RVZ_HIP(hipStreamSynchronize(e->stream), e);
    double sum[2] = {0.0, 0.0};
    int32_t n[2] = {0, 0};
    for (const auto& mk : e->ev_marks) {
        float ms = 0.0f;
        RVZ_HIP(hipEventElapsedTime(&ms, e->ev_pool[mk.second], e->ev_pool[mk.second + 1]), e);
        sum[mk.first] += ms;
        n[mk.first] += 1;
    }
    for (int k = 0; k < 2; ++k) {
        out_ms[k] = n[k] ? sum[k] / n[k] : 0.0;
        out_n[k] = n[k];
    }
    return RVZ_OK;
}

int rvz_tree_nodes(const rvz_engine* e) { return e ? e->M : RVZ_EINVAL; }

int rvz_tree_export(rvz_engine* e, void* nodes_out, uint32_t* meta_out) {
    if (!e) return RVZ_EINVAL;
    int r = flush_pending(e);
    if (r != RVZ_OK) return r;
    const size_t n = (size_t)e->v.G * e->M;
    if (nodes_out) RVZ_HIP(hipMemcpyAsync(nodes_out, e->v.nodes, n * sizeof(Node), hipMemcpyDeviceToDevice, e->stream), e);
    if (meta_out) RVZ_HIP(hipMemcpyAsync(meta_out, e->v.meta, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, e->stream), e);
    return RVZ_OK;
}

int rvz_footprint(const rvz_engine* e, int64_t* bytes_tree, int64_t* bytes_env) {
    if (!e) return RVZ_EINVAL;
    const int64_t G = e->v.G;
    if (bytes_tree)
        *bytes_tree = G * e->M * (int64_t)(sizeof(Node) + sizeof(uint32_t)) +
                      G * (PATH_CAP * 4 + 4 * 4 + 8) + G * (4 + 2 * e->E * 4);   // + memo
    if (bytes_env) *bytes_env = G * (8 + 8 + 16) + G * (RNG_DRAWS * 8 + 4);
    return RVZ_OK;
}

}  // extern "C"
