// rvz_play.hip.h — fused self-play (rvz_play): a workgroup plays its own games, search and leaf
// evaluation in one persistent launch. Included by csrc/rvz_engine.hip inside its anonymous
// namespace, after the search device functions (select_phase, expand_backup_phase, act_game,
// reset_game); the evaluator device functions come from rvz_h2.hip.h (h2_pass) and
// rvz_resnet_common.hip.h (heads_fc16).
//
// The ply loop of SelfPlayRunner (per batch: k_step, the h2 trunk, the FC heads; then k_act and
// k_autoreset, self_play.py:80-101 with mcts.py:322-407 and :642-694) as one launch:
// workgroup w owns games [w * gpw, (w + 1) * gpw) and alternates
//  * a search phase: one wave per game (four games at a time) runs the pending expand + the next
//    batch's selection, or, after the last batch, act + autoreset, until the game has queued its
//    next NN row or has committed `plies` plies in this launch;
//  * an evaluation phase: the queued rows in NBOARD-board passes of the h2 trunk (h2_pass, the
//    code of k_resnet_h2) and 16-board passes of the FC heads (heads_fc16, as k_heads_mfma).
// Each per-game computation is the one the unfused launches make, and an h2 row's outputs depend
// only on its position (test_h2_live_rows), so the games are bit-identical to SelfPlayRunner's
// (tests/test_gpu_play.py). Inside a ply there is no kernel boundary, launch ramp or tail: the
// two workgroups on a CU overlap one's search phase with the other's trunk passes.

struct PlayArgs {
    const float* prm;
    Layout L;
    const uint16_t* blob;
    int n_blocks;
    float* x;          // [G][3][NSQ] the queued rows' leaf planes (select_phase, row = game)
    int32_t* need;     // [G] queued copies (select_phase)
    float* work;       // [G][192] 1x1 head-conv outputs
    float* logits;     // [G][NPOL]
    float* value;      // [G]
    float* ovf;        // sticky f16-overflow word of the evaluator, or null
    int gpw, plies, skip_last, reset, S, B;
    double temperature;
    int64_t* seeds;
    int64_t stride;
    int64_t* ply_ctr;  // [G] committed plies per slot
    int64_t* done;     // [G] finished games per slot
    int32_t* out_idx;  // [G] the last act's index
    double* out_p;     // [G][NPOL] the last act's policy vector
    int32_t* hist;     // [plies][G] every act's index in this launch, or null
    unsigned long long* rows;   // += the rows this launch evaluated, or null
    const int32_t* budget;      // [G] plies game g commits in this launch (<= plies), or null
    unsigned spin_limit;        // queue waits give up (ERR_SCHED) after this many sleeps
    // the cross-game NN-output table (rvz_play_table; tab null: off)
    unsigned long long* tab;    // [slots][TabGeo<BS>::STRIDE] granules {value, tag = generation}
    unsigned* tclaim;           // [slots] the generation that claimed the slot
    const unsigned* tgen;       // the current generation (device word, >= 1)
    unsigned tmask;             // slots - 1
    int tmaxd;                  // positions with at most this many discs are looked up / stored
    unsigned long long* tstats; // += {hits, inserts}, or null
    // self-play records (or null): the position before each committed act and its policy vector,
    // [plies][G] (rec_p [plies][G][NPOL]); hist holds the act's index
    uint64_t* rec_black;
    uint64_t* rec_white;
    int32_t* rec_side;
    double* rec_p;
    // schedule. Static (q_next null): workgroup w owns game group w for all `plies` plies.
    // Queue: tasks t = (group t % n_groups, ply t / n_groups) drawn in order from q_next; a
    // group's ply p starts after q_done[group] reached p (its ply p-1 published: agent-scope
    // release by the workgroup that played it, acquire by the next). Both zeroed per launch.
    unsigned* q_next;
    unsigned* q_done;  // [n_groups]
    int n_groups;
    // the per-XCD pass gate (play_gate; gate null or gate_frac 0: off): [8][16] words, one
    // 128-byte line per XCD, zeroed per launch with the queue words
    unsigned long long* gate;
    unsigned gate_frac;  // a round opens when this fraction (Q16) of the XCD's running workgroups
                         // arrived,
    unsigned gate_t;     // or this long after a waiter's arrival (s_memrealtime ticks, 100 MHz);
    unsigned gate_late;  // a workgroup arriving this soon after a round opened joins it at once
};
constexpr int PLAY_GPW_MAX = 64;
// the 8x8 / 64-filter (C2) geometry keeps its head-conv rows in LDS for the FC heads (no
// workspace round trip): at most 8 games per workgroup, so that 8 rows of LDS hold a cycle's rows
template <int F, int BS>
__host__ __device__ constexpr bool play_heads_lds() { return F == 64 && BS == 8; }
template <int F, int BS>
__host__ __device__ constexpr int play_gpw_max() {
    return play_heads_lds<F, BS>() ? 8 : PLAY_GPW_MAX;
}
// game flags: a row queued for the NN, its output ready for the expand, the game's plies done,
// its row in this cycle's passes, its row held back last cycle (an odd row waits one cycle)
enum : int { PF_QUEUED = 1, PF_READY = 2, PF_DONE = 4, PF_EVAL = 8, PF_HELD = 16 };
constexpr int32_t ERR_SCHED = 16;   // a queue wait timed out (device error word)

// ---- the cross-game NN-output table (rvz_play_table) ---------------------------------------
// An h2 row's outputs depend only on its input planes (test_h2_live_rows), and the planes are a
// function of three bitboards (mover, opponent, the mover's legal moves: get_canonical_state,
// game.py:131-162). So a row evaluated once — by any game, in any earlier cycle, with the same
// weights — can stand in for a new evaluation of the same (P, O, V): its logits and value are
// bitwise what the trunk and heads would return. The opening positions repeat across games
// (tools/exp_xgame.py: 11.9% of the C2 headline's rows repeat an earlier row's position).
// Slot layout: NG = NSQ + 8 granules of 8 bytes {32-bit datum, 32-bit tag}: logits 0..NSQ-1, the
// pass logit (NSQ), the value (NSQ + 1), the key words P lo/hi, O lo/hi, V lo/hi (NSQ + 2 ..).
// Every granule is stored whole by one agent-scope 8-byte store and read by agent-scope 8-byte
// loads (MI355X_MICROARCH.md R2 granules: the data is its own flag, no fence): a reader accepts
// a slot only if every granule carries the current generation as its tag and the key matches;
// a slot being written, empty, or of an older generation fails the tag check (a miss, never a
// wrong row). A slot is claimed once per generation by a compare-and-swap of its claim word, so
// all granules tagged with a generation were written by that generation's one claimant; a new
// generation (new weights: rvz_search_memo_reset, or another weight blob) invalidates every slot
// without touching the table.
template <int BS>
struct TabGeo {
    static constexpr int NSQ = Geo<BS>::NSQ;
    static constexpr int NG = NSQ + 8;
    static constexpr int STRIDE = (NG + 7) / 8 * 8;   // granules per slot (64-byte multiple)
};
constexpr int TAB_PROBES = 8;

__device__ __forceinline__ uint64_t tab_mix(uint64_t z) {
    z ^= z >> 30;
    z *= 0xbf58476d1ce4e5b9ull;
    z ^= z >> 27;
    z *= 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t tab_hash(uint64_t P, uint64_t O, uint64_t V) {
    return tab_mix(P ^ tab_mix(O ^ tab_mix(V + 0x9e3779b97f4a7c15ull)));
}
// the datum of granule idx of a slot holding (P, O, V) with this row / value (key part only
// when row is null)
template <int NSQ>
__device__ __forceinline__ uint32_t tab_key_word(int idx, uint64_t P, uint64_t O, uint64_t V) {
    const int k = idx - (NSQ + 2);
    const uint64_t w = k < 2 ? P : (k < 4 ? O : V);
    return (k & 1) ? (uint32_t)(w >> 32) : (uint32_t)w;
}

// Loads slot `sl`'s granules (lane l: granules l and 64 + l) and checks tags and key: returns
// 0 if some granule is not of generation `gen` (empty, being written, older), 1 if the slot is a
// whole slot of this generation holding another key, 2 if it holds (P, O, V).
template <int BS>
__device__ __forceinline__ int tab_read(const unsigned long long* __restrict__ tab, uint32_t sl,
                                         uint32_t gen, uint64_t P, uint64_t O, uint64_t V,
                                         int lane, uint64_t& x0, uint64_t& x1) {
    using T = TabGeo<BS>;
    constexpr int NSQ = T::NSQ, NG = T::NG;
    const unsigned long long* e = tab + (size_t)sl * T::STRIDE;
    x0 = 0;
    x1 = 0;
    if (lane < NG) x0 = __hip_atomic_load(e + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (NG > 64 && lane < NG - 64)
        x1 = __hip_atomic_load(e + 64 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    bool stale = false, other = false;
    if (lane < NG) {
        stale |= (uint32_t)(x0 >> 32) != gen;
        if (lane >= NSQ + 2) other |= (uint32_t)x0 != tab_key_word<NSQ>(lane, P, O, V);
    }
    if (NG > 64 && lane < NG - 64) {
        stale |= (uint32_t)(x1 >> 32) != gen;
        if (64 + lane >= NSQ + 2) other |= (uint32_t)x1 != tab_key_word<NSQ>(64 + lane, P, O, V);
    }
    if (__ballot(stale) != 0ull) return 0;
    return __ballot(other) != 0ull ? 1 : 2;
}

// granule idx's datum, wave-uniform (idx a compile-time constant >= NSQ)
template <int BS, int IDX>
__device__ __forceinline__ uint32_t tab_datum(uint64_t x0, uint64_t x1) {
    if constexpr (IDX < 64) return (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x0, IDX);
    else return (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x1, IDX - 64);
}

// A hit writes the stored row into the game's logits / value rows (as the FC heads would) and
// returns true. Probes stop at the first slot that is not a valid slot of this generation.
template <int BS>
__device__ __forceinline__ bool tab_lookup(const PlayArgs& a, uint32_t gen, uint64_t P,
                                           uint64_t O, uint64_t V, int lane, int g) {
    constexpr int NSQ = Geo<BS>::NSQ, NPOL = Geo<BS>::NPOL;
    const uint64_t h = tab_hash(P, O, V);
    for (int i = 0; i < TAB_PROBES; ++i) {
        const uint32_t sl = (uint32_t)(h + i) & a.tmask;
        uint64_t x0, x1;
        const int r = tab_read<BS>(a.tab, sl, gen, P, O, V, lane, x0, x1);
        if (r == 0) return false;   // not a whole slot of this generation: the chain ends
        if (r == 1) continue;       // another key's slot: probe on
        float* row = a.logits + (size_t)g * NPOL;
        if (lane < NSQ) row[lane] = __uint_as_float((uint32_t)x0);
        if (lane == 0) {
            row[NSQ] = __uint_as_float(tab_datum<BS, NSQ>(x0, x1));
            a.value[g] = __uint_as_float(tab_datum<BS, NSQ + 1>(x0, x1));
        }
        return true;
    }
    return false;
}

// Stores game g's evaluated row (a.logits / a.value, written by the FC heads of this
// workgroup) for (P, O, V). Returns 1 if this wave wrote a slot.
template <int BS>
__device__ __forceinline__ int tab_insert(const PlayArgs& a, uint32_t gen, uint64_t P, uint64_t O,
                                          uint64_t V, int lane, int g) {
    using T = TabGeo<BS>;
    constexpr int NSQ = T::NSQ, NPOL = Geo<BS>::NPOL, NG = T::NG;
    const uint64_t h = tab_hash(P, O, V);
    for (int i = 0; i < TAB_PROBES; ++i) {
        const uint32_t sl = (uint32_t)(h + i) & a.tmask;
        uint32_t c = 0;
        if (lane == 0) c = __hip_atomic_load(a.tclaim + sl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        c = (uint32_t)__builtin_amdgcn_readfirstlane((int)c);
        if (c == gen) {   // taken in this generation: ours already, or another key's
            uint64_t x0, x1;
            if (tab_read<BS>(a.tab, sl, gen, P, O, V, lane, x0, x1) == 2) return 0;
            continue;
        }
        uint32_t won = 0;
        if (lane == 0) {
            uint32_t expect = c;
            won = __hip_atomic_compare_exchange_strong(a.tclaim + sl, &expect, gen,
                                                       __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT) ? 1u : 0u;
        }
        if (!__builtin_amdgcn_readfirstlane((int)won)) continue;
        const float* row = a.logits + (size_t)g * NPOL;
        const float val = a.value[g];
        unsigned long long* e = a.tab + (size_t)sl * T::STRIDE;
        const unsigned long long tag = (unsigned long long)gen << 32;
        if (lane < NG) {
            const uint32_t d = lane < NPOL ? __float_as_uint(row[lane])
                               : lane == NSQ + 1 ? __float_as_uint(val)
                                                 : tab_key_word<NSQ>(lane, P, O, V);
            __hip_atomic_store(e + lane, tag | d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (NG > 64 && lane < NG - 64) {
            const int idx = 64 + lane;
            const uint32_t d = idx < NPOL ? __float_as_uint(row[idx])
                               : idx == NSQ + 1 ? __float_as_uint(val)
                                                : tab_key_word<NSQ>(idx, P, O, V);
            __hip_atomic_store(e + idx, tag | d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return 1;
    }
    return 0;
}

// ---- the per-XCD pass gate (rvz_play_gate; 8x8 at 128 and 256 filters) ---------------------
// At 10x128 every trunk pass streams the whole 11.8 MB of f16-pair weights, and the 64 workgroups
// of an XCD, each at its own layer, keep all of it live in a 4 MB L2 (45% L2 hits,
// the fabric path full, the clock held at 1.55 GHz). The gate makes a workgroup about to start a
// pass wait until a fraction of its XCD's running workgroups have arrived (or a timeout), so the
// XCD's passes start in one cohort whose members read the same layer's weights at the same time;
// a workgroup arriving shortly after a round opened (a search phase made it late) joins that
// cohort at once instead of waiting for the next. Timing only: the games do not depend on it. One
// lane; no data is handed over, so no fences. At 256 filters (47 MB per pass at 10 blocks, one
// workgroup per CU) the same cohorts are worth +10%.
// An XCD's line: word 0 {round:32 | arrivals:32}, word 1 when the current round opened
// (s_memrealtime), word 2 the XCD's running workgroups of this launch.
__device__ __forceinline__ void gate_open(unsigned long long* w, unsigned r) {
    unsigned long long v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while ((unsigned)(v >> 32) == r) {
        if (__hip_atomic_compare_exchange_strong(w, &v, (unsigned long long)(r + 1u) << 32,
                                                 __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)) {
            __hip_atomic_store(w + 1, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
    }
}
__device__ __forceinline__ unsigned long long* gate_line(unsigned long long* gate) {
    const unsigned x = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20) & 7u;   // XCC_ID
    return gate + 16 * x;
}
// a workgroup starts (+1) / ends (-1) its part of the launch on this XCD
__device__ __forceinline__ void gate_running(unsigned long long* gate, long long d) {
    __hip_atomic_fetch_add(gate_line(gate) + 2, (unsigned long long)d, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void play_gate(unsigned long long* gate, unsigned frac, unsigned t,
                                          unsigned late) {
    unsigned long long* w = gate_line(gate);
    if (late) {   // the round that opened moments ago: join its cohort without an arrival
        const unsigned long long t_open =
            __hip_atomic_load(w + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (t_open && __builtin_amdgcn_s_memrealtime() - t_open < late) return;
    }
    const unsigned long long running =
        __hip_atomic_load(w + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // a few workgroups per XCD (a small launch, or a launch's tail) share the L2 without help:
    // no cohort to wait for
    if (running < 4) return;
    const unsigned k = max(1u, (unsigned)((running * frac) >> 16));
    const unsigned long long old =
        __hip_atomic_fetch_add(w, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned r = (unsigned)(old >> 32);
    if ((unsigned)old + 1u >= k) {
        gate_open(w, r);
        return;
    }
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        __builtin_amdgcn_s_sleep(2);
        const unsigned long long v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((unsigned)(v >> 32) != r) return;
        if (__builtin_amdgcn_s_memrealtime() - t0 > t) {
            gate_open(w, r);
            return;
        }
    }
}

struct PlayCtx {
    View v;
    PlayArgs a;
};
// The launch's arguments, re-read from the kernarg segment at each use site: `play_ctx()` hides
// the kernarg pointer from the optimiser (an empty asm), so the fields a phase reads are loaded
// (s_load, scalar cache) inside that phase instead of being hoisted to the kernel entry and held
// in SGPRs across the trunk passes (~100 SGPRs of View + PlayArgs: spills).
// The thread index made opaque at the head of a phase: address arithmetic derived from it is
// recomputed in that phase instead of being hoisted out of the ply loop and held in registers
// across the other phases (the trunk, the search and the heads each need most of the registers)
__device__ __forceinline__ int opaque_tid() {
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}
__device__ __forceinline__ const PlayCtx& play_ctx() {
    const __attribute__((address_space(4))) char* p =
        (const __attribute__((address_space(4))) char*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return *(const PlayCtx*)p;
}

// RVZ_PLAY_TIMING (tools/exp_play_phases.py, instrumented builds only): per workgroup, shader
// clocks (s_memtime) spent in [0] the search phase (to its barrier), [1] the trunk passes,
// [2] the FC heads, [3] the whole launch; [4] cycles of the loop, [5] trunk passes, [6] rows,
// [7] the workgroup's XCC / CU (HW_ID); [8] cycles waiting for a task's previous ply (queue),
// [9] tasks, [10] the launch clock at the workgroup's end (s_memrealtime, 100 MHz)
#ifdef RVZ_PLAY_TIMING
__device__ unsigned long long g_play_t[16384][12];
#define PT_NOW(t) const unsigned long long t = __builtin_amdgcn_s_memtime()
#define PT_ADD(i, v) if (tid == 0 && blockIdx.x < 16384) g_play_t[blockIdx.x][i] += (v)
#else
#define PT_NOW(t)
#define PT_ADD(i, v)
#endif

// Rejected schedule / phase variants (measured, not kept: dealing the search phase's games
// round-robin, the last ply split into half tasks, the FC heads' weights loaded before the last
// pass's head convs, s_setprio for the tower) are patches in tools/patches/ (README there).
template <int F, int NBOARD, int CTW, int PTW, int BS, int OCC>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC, OCC)))
void k_play(PlayCtx ctx0) {
    (void)ctx0;   // read through play_ctx()
    using WT = WaveTilesH<F, CTW, PTW>;
    constexpr bool ILV = RVZ_H2_ILV && NBOARD == 2 && BS == 8 && PTW == 4 && WT::CG == 2;
    using GH = GeoH<NBOARD, BS, 64 * CTW * H2_TM / F, ILV>;
    using C = CfgH<F, GH::NPIX>;
    constexpr int NPOL = Geo<BS>::NPOL;
    constexpr bool HLDS = play_heads_lds<F, BS>();
    constexpr int GMAX = play_gpw_max<F, BS>();
    constexpr int HROW = heads_in_floats(BS) / 16;
    // LDS: the trunk's activation image; between passes its head holds the search phase's act /
    // reset scratch (per wave) or (not HLDS) the FC heads' input rows
    constexpr int SP_BYTES = WPB * (NPOL + 7) * 8;
    // the search phase's act / reset scratch and the FC heads' rows live in the activation image
    // only: below C::RMAX, so they never overlap the range maxima / overflow words (RangeLds),
    // which are pass-local
    static_assert(heads_in_floats(BS) * 4 <= C::RMAX, "heads rows fit");
    static_assert(SP_BYTES + WPB * 624 * 4 <= C::RMAX, "act / reset scratch fits");
    __shared__ __attribute__((aligned(16))) char smem[C::BYTES];
    __shared__ int st_k[GMAX];   // next batch of the game's search (E: act next)
    __shared__ int st_f[GMAX];   // PF_* flags
    __shared__ int st_p[GMAX];   // plies committed in this launch
    __shared__ uint64_t st_bits[GMAX * 3];              // the queued leaf's (P, O, V) per game
    __shared__ uint64_t q_bits[(GMAX + NBOARD) * 3];    // the same, in this cycle's row order
    __shared__ __attribute__((aligned(16))) float hin[HLDS ? GMAX * HROW : 4];   // heads rows
    __shared__ int q_rows[GMAX + 16];
    __shared__ int s_nq;
    __shared__ float vpart[4][16];
    __shared__ int s_task[2];
    __shared__ unsigned s_tgen;
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    int E, G, gpw, total, queue, task_plies;
    {
        const PlayCtx& c = play_ctx();
        E = c.v.E;
        G = c.v.G;
        gpw = c.a.gpw;
        queue = c.a.q_next != nullptr;
        total = queue ? c.a.n_groups * c.a.plies : 0;
        task_plies = queue ? 1 : c.a.plies;
    }
    bool ovf = false;
    // the workgroup's rows, table hits and inserts, in LDS (no registers held across the phases)
    __shared__ unsigned s_cnt[3];
    if (tid < 3) s_cnt[tid] = 0u;
    if (tid == 0) {
        const PlayArgs& a = play_ctx().a;
        s_tgen = a.tab ? __hip_atomic_load(a.tgen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    }
    double* sp = reinterpret_cast<double*>(smem) + wave * (NPOL + 7);
    uint32_t* key = reinterpret_cast<uint32_t*>(smem + SP_BYTES) + wave * 624;
    if constexpr (F >= 128 && BS == 8) {   // the pass gate counts the XCD's running workgroups
        const PlayArgs& a = play_ctx().a;
        if (tid == 0 && a.gate_frac > 0) gate_running(a.gate, 1);
    }
    PT_NOW(t_start);
    for (int task_i = 0;; ++task_i) {
        // ---- the next task: a game group and the ply it starts at
        int gi, ply0;
        if (!queue) {
            if (task_i > 0) break;
            gi = blockIdx.x;
            ply0 = 0;
        } else {
            PT_NOW(t_q0);
            if (tid == 0) {
                const PlayCtx& c = play_ctx();
                const PlayArgs& a = c.a;
                // once a wait timed out (ERR_SCHED) no workgroup draws another task: the launch
                // drains, and the engine state is undefined until the games are reset (rvz.h)
                const bool failed = __hip_atomic_load(c.v.err, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT) & ERR_SCHED;
                const unsigned t =
                    failed ? (unsigned)total
                           : __hip_atomic_fetch_add(a.q_next, 1u, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
                int tg = -1, tp = 0;
                if ((int)t < total) {
                    tg = (int)(t % (unsigned)a.n_groups);
                    tp = (int)(t / (unsigned)a.n_groups);
                    // the group's previous ply: played (and published) by the workgroup that
                    // drew it n_groups tasks ago, which is running; bounded spin, abandoned as
                    // soon as another workgroup's wait timed out
                    unsigned spins = 0;
                    while ((int)__hip_atomic_load(a.q_done + tg, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT) < tp) {
                        __builtin_amdgcn_s_sleep(4);
                        ++spins;
                        if (spins > a.spin_limit ||
                            ((spins & 1023u) == 0 &&
                             (__hip_atomic_load(c.v.err, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT) & ERR_SCHED))) {
                            atomicOr(c.v.err, ERR_SCHED);
                            tg = -1;
                            break;
                        }
                    }
                    // ONE acquire after the match
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                s_task[0] = tg;
                s_task[1] = tp;
            }
            __syncthreads();   // the other waves load the group's state after the acquire
            gi = __builtin_amdgcn_readfirstlane(s_task[0]);
            ply0 = __builtin_amdgcn_readfirstlane(s_task[1]);
            if (gi < 0) break;
            PT_NOW(t_q1);
            PT_ADD(8, t_q1 - t_q0);
            PT_ADD(9, 1);
        }
        const int g0 = gi * gpw;
        const int ng = min(gpw, G - g0);
        {   // a game whose ply budget this task's ply reaches starts done
            const int32_t* bud = play_ctx().a.budget;
            for (int j = tid; j < ng; j += 256) {
                st_k[j] = 0;
                st_f[j] = (bud && ply0 >= bud[g0 + j]) ? PF_DONE : 0;
                st_p[j] = 0;
            }
        }
        __syncthreads();
        for (;;) {
            PT_NOW(t_c0);
            // search phase: each game not waiting for its row advances until it queues the next
            // row or has committed its plies (wave-uniform control flow per game)
            for (int j = wave; j < ng; j += WPB) {
                const PlayCtx& c = play_ctx();
                const View& v = c.v;
                const PlayArgs& a = c.a;
                const int lane = opaque_tid() & 63;
                const int g = g0 + j;
                int f = __builtin_amdgcn_readfirstlane(st_f[j]);
                if (f & (PF_QUEUED | PF_DONE)) continue;
                int k = __builtin_amdgcn_readfirstlane(st_k[j]);
                int np = __builtin_amdgcn_readfirstlane(st_p[j]);
                WT_NOW(ft_step);
                FT_CNT();
                for (;;) {
                    unsigned long long ab = 0;
                    if (k < E) {   // k_step: the pending expand + backup, then batch k's selection
                        const int first = k == 0;
                        const GameS root = load_game(v, g);
                        uint32_t root_meta = 0, carry = LINK_NONE;
                        int root_n = 0;
                        if (!first) {
                            root_meta = v.meta[(size_t)g * v.M];
                            root_n = v.nodes[(size_t)g * v.M].n;
                        } else if (v.memo) {
                            carry = v.carry[g];
                        }
                        if (f & PF_READY) {
                            WT_NOW(ft_e);
                            const ExpIn x = expand_load<BS>(v, g, lane, a.logits, a.value);
                            const int rn =
                                expand_backup_phase<BS>(v, g, lane, x, 1, &root_meta, ab);
                            if (rn >= 0) root_n = rn;
                            f &= ~PF_READY;
                            FT_ADD(0, ft_e);
                        }
                        const int bsz = min(a.B, a.S - k * a.B);
                        const int copies = select_phase<BS, float>(v, g, lane, first, bsz, k, root,
                                                                   root_meta, root_n, carry, a.x,
                                                                   a.need, ab, st_bits + 3 * j);
                        ++k;
                        // the last batch's row with skip_last: left unevaluated (rvz_search_skip)
                        if (copies > 0 && !(k == E && a.skip_last)) {
                            if (a.tab) {   // an earlier evaluation of this position: no new row
                                const uint64_t P = st_bits[3 * j], O = st_bits[3 * j + 1],
                                               Vb = st_bits[3 * j + 2];
                                WT_NOW(ft_t);
                                const bool hit = __popcll(P | O) <= a.tmaxd &&
                                                 tab_lookup<BS>(a, s_tgen, P, O, Vb, lane, g);
                                WT_ADD(0, ft_t);
                                if (hit) {
                                    // the expand reads the row (and select's pend / path words)
                                    // back in this wave
                                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
                                    f |= PF_READY;
                                    if (lane == 0) atomicAdd(&s_cnt[1], 1u);
                                    continue;
                                }
                            }
                            f |= PF_QUEUED;
                            break;
                        }
                        continue;
                    }
                    // k_act: the last batch's expand (or visit-count backup), the action, the move
                    WT_NOW(ft_a);
                    bool over = false;
                    double* outp = a.out_p;
                    if (a.rec_black) {   // the record of this ply: the position before the move
                        const size_t ri = (size_t)(ply0 + np) * v.G + g;
                        if (lane == 0) {
                            a.rec_black[ri] = v.black[g];
                            a.rec_white[ri] = v.white[g];
                            a.rec_side[ri] = v.status[(size_t)g * 4];
                        }
                        outp = a.rec_p + (size_t)(ply0 + np) * v.G * Geo<BS>::NPOL;
                    }
                    const int idx = act_game<BS>(v, g, lane, sp, (f & PF_READY) ? 1 : 2,
                                                 a.logits, 1, a.value, a.temperature, nullptr, 1,
                                                 a.out_idx, outp, &over);
                    f &= ~PF_READY;
                    // k_autoreset: count the ply; a finished game restarts with its slot's next
                    // seed
                    int64_t sd = 0;
                    if (lane == 0) {
                        if (idx >= 0) a.ply_ctr[g] += 1;
                        if (a.hist) a.hist[(size_t)(ply0 + np) * v.G + g] = idx;
                        if (a.reset && over) {
                            a.done[g] += 1;
                            sd = a.seeds[g] + a.stride;
                            a.seeds[g] = sd;
                        }
                    }
                    if (a.reset && over) {
                        sd = __shfl(sd, 0);
                        reset_game<BS>(v, g, lane, (uint32_t)(sd & 0xFFFFFFFFll), key);
                    }
                    FT_ADD(1, ft_a);
                    ++np;
                    k = 0;
                    if (np >= task_plies || (a.budget && ply0 + np >= a.budget[g])) {
                        f |= PF_DONE;
                        break;
                    }
                }
                FT_ADD(2, ft_step);
                if (lane == 0) {
                    st_k[j] = k;
                    st_f[j] = f;
                    st_p[j] = np;
                }
            }
            __syncthreads();
            PT_NOW(t_c1);
            PT_ADD(0, t_c1 - t_c0);
            PT_ADD(4, 1);
            if (tid == 0) {   // the queued rows, in game order
                int n = 0;
                for (int j = 0; j < ng; ++j)
                    if (st_f[j] & PF_QUEUED) ++n;
                // rows that would leave the last pass partly empty wait one cycle (their games
                // sit out one search phase: a game's computation is the same whichever cycle
                // evaluates its row), unless they waited last cycle or there is no full pass
                int hold = n > NBOARD ? n % NBOARD : 0;
                for (int j = ng - 1; j >= 0; --j) {
                    const int fj = st_f[j];
                    if (!(fj & PF_QUEUED)) continue;
                    if (hold > 0 && !(fj & PF_HELD)) {
                        st_f[j] = fj | PF_HELD;
                        --hold;
                    } else {
                        st_f[j] = (fj & ~PF_HELD) | PF_EVAL;
                    }
                }
                n = 0;
                for (int j = 0; j < ng; ++j)
                    if (st_f[j] & PF_EVAL) {
                        for (int ch = 0; ch < 3; ++ch) q_bits[3 * n + ch] = st_bits[3 * j + ch];
                        q_rows[n++] = g0 + j;
                    }
                for (int i = n; i < n + 16; ++i) q_rows[i] = -1;
                for (int i = 3 * n; i < 3 * (n + NBOARD); ++i) q_bits[i] = 0;
                s_nq = n;
            }
            __syncthreads();
            const int nq = __builtin_amdgcn_readfirstlane(s_nq);
            if (nq == 0) break;   // every game has committed its plies
            if (tid == 0) s_cnt[0] += (unsigned)nq;
            PT_NOW(t_c2);

            // evaluation phase: the trunk over the queued rows, NBOARD boards per pass
            for (int p0 = 0; p0 < nq; p0 += NBOARD) {
                // the per-XCD pass gate (rvz_play_gate: on by default; built into the 8x8 forms
                // at 128 and 256 filters)
                if constexpr (F >= 128 && BS == 8) {
                    if (play_ctx().a.gate_frac > 0) {
                        if (tid == 0) {
                            const PlayArgs& a = play_ctx().a;
                            play_gate(a.gate, a.gate_frac, a.gate_t, a.gate_late);
                        }
                        __syncthreads();
                    }
                }
                const PlayArgs& a = play_ctx().a;
                int gb[NBOARD];
#pragma unroll
                for (int k = 0; k < NBOARD; ++k) gb[k] = q_rows[p0 + k];
                const int t = opaque_tid();
                if constexpr (HLDS)
                    h2_pass<F, NBOARD, CTW, PTW, BS>(
                        smem, a.x, gb, q_bits + 3 * p0, a.prm, a.L, a.blob, a.n_blocks,
                        HeadsInLds<BS>{hin, p0, nq}, t, t & 63,
                        __builtin_amdgcn_readfirstlane(t >> 6), ovf);
                else
                    h2_pass<F, NBOARD, CTW, PTW, BS>(
                        smem, a.x, gb, q_bits + 3 * p0, a.prm, a.L, a.blob, a.n_blocks,
                        HeadsGlobalIdx<NBOARD>(a.work, gb), t, t & 63,
                        __builtin_amdgcn_readfirstlane(t >> 6), ovf);
                __syncthreads();
            }
            PT_NOW(t_c3);
            PT_ADD(1, t_c3 - t_c2);
            PT_ADD(5, (nq + NBOARD - 1) / NBOARD);
            PT_ADD(6, nq);
            for (int h0 = 0; h0 < nq; h0 += 16) {
                const PlayArgs& a = play_ctx().a;
                if constexpr (HLDS)   // the rows are in hin already (HeadsInLds); columns >= 8 mirror 0-7
                    heads_fc16<BS, HeadRowsList, false, false, GMAX>(
                        a.work, HeadRowsList{q_rows + h0}, a.prm, a.L, a.logits, a.value, hin,
                        vpart, opaque_tid());
                else
                    heads_fc16<BS, HeadRowsList, false, true>(
                        a.work, HeadRowsList{q_rows + h0}, a.prm, a.L, a.logits, a.value,
                        reinterpret_cast<float*>(smem), vpart, opaque_tid());
            }
            if (play_ctx().a.tab) {   // store the new rows of table positions (one wave per row)
                __syncthreads();      // the heads' logits / value rows are written
                for (int i = wave; i < nq; i += WPB) {
                    const PlayArgs& a = play_ctx().a;
                    const uint64_t P = q_bits[3 * i], O = q_bits[3 * i + 1], Vb = q_bits[3 * i + 2];
                    if (__popcll(P | O) <= a.tmaxd)
                        if (tab_insert<BS>(a, s_tgen, P, O, Vb, opaque_tid() & 63, q_rows[i]) &&
                            (opaque_tid() & 63) == 0)
                            atomicAdd(&s_cnt[2], 1u);
                }
            }
            for (int j = tid; j < ng; j += 256)
                if (st_f[j] & PF_EVAL) st_f[j] = (st_f[j] & ~(PF_QUEUED | PF_EVAL)) | PF_READY;
            __syncthreads();
            PT_NOW(t_c4);
            PT_ADD(2, t_c4 - t_c3);
        }
        if (queue) {   // publish the group's ply: every wave drained, then ONE agent release + flag
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_store(play_ctx().a.q_done + gi, (unsigned)(ply0 + 1), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    if constexpr (F >= 128 && BS == 8) {   // no more passes from this workgroup
        const PlayArgs& a = play_ctx().a;
        if (tid == 0 && a.gate_frac > 0) gate_running(a.gate, -1);
    }
#ifdef RVZ_PLAY_TIMING
    {
        PT_NOW(t_end);
        PT_ADD(3, t_end - t_start);
        if (tid == 0 && blockIdx.x < 16384)
            g_play_t[blockIdx.x][10] = __builtin_amdgcn_s_memrealtime();
        if (tid == 0 && blockIdx.x < 16384)
            g_play_t[blockIdx.x][7] =
                ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) |
                __builtin_amdgcn_s_getreg((31 << 11) | 4);
    }
#endif
    float* ovw = play_ctx().a.ovf;
    if (ovf && ovw) *ovw = 1.0f;   // benign race: every writer stores 1
    unsigned long long* rows = play_ctx().a.rows;
    __syncthreads();                       // every wave's counts are in
    if (rows && tid == 0) atomicAdd(rows, (unsigned long long)s_cnt[0]);
    unsigned long long* ts = play_ctx().a.tstats;
    if (ts && tid == 0) {          // the workgroup's hits and inserts
        if (s_cnt[1]) atomicAdd(ts, (unsigned long long)s_cnt[1]);
        if (s_cnt[2]) atomicAdd(ts + 1, (unsigned long long)s_cnt[2]);
    }
}
