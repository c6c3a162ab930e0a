// rvz_play12.hip.h — the fused self-play launch with specialised teams (RVZ_PLAY_TEAMS, the C2
// geometry: 8x8, 64 filters, two boards per trunk pass). Included by csrc/rvz_engine.hip after
// rvz_play.hip.h, inside its anonymous namespace.
//
// k_play (rvz_play.hip.h) runs two 4-wave workgroups per CU; each alternates its games' search
// phase, its trunk passes and its FC heads, so a SIMD holds two tower waves only while both
// workgroups are in their towers (the MFMA pipes are busy 73% of the launch).
// k_play12 is one 12-wave workgroup per CU, three teams of four waves (one wave per SIMD each):
//  * trunk teams T0, T1: take the queued leaf rows two at a time from an LDS ring and run the h2
//    trunk pass on them (h2_pass with the H2Diet knobs: three waves per SIMD fit in 168 VGPRs),
//    writing the 1x1 head-conv rows into the FC heads' LDS input;
//  * search team S: plays the tasks of two slots (each a group of <= 8 games for one ply, drawn
//    from the queue of k_play): while the trunk teams evaluate one slot's rows it runs the other
//    slot's search phase (the pending expands and the next selections, acts, autoresets, table
//    lookups), then the FC heads of a slot whose rows are all done and its table inserts.
// Each game's computation is the one k_play makes (the same device functions, in the same order
// per game); a row's outputs do not depend on which rows share its pass or heads column
// (test_h2_live_rows), so the games are those of k_play built with the same trunk knobs.
// Teams synchronise with 4-wave barriers on LDS counters (gfx950 has one workgroup barrier) and
// hand rows over through LDS words; every wait is bounded (ERR_SCHED, then every team exits).

#ifndef RVZ_PLAY_TEAMS
#define RVZ_PLAY_TEAMS 0      // rvz_play runs k_play12 for the C2 geometry (env RVZ_PLAY_TEAMS)
#endif

#ifndef RVZ_T12_SLOTS
#define RVZ_T12_SLOTS 2
#endif
// the trunk teams' knobs (<= 168 VGPRs): 0 H2Diet (no activation prefetch, weights 1 k-step
// ahead); 1 activation prefetch 1, weights 1 ahead, epilogue operands loaded late; 2 no activation
// prefetch, weights 2 ahead, epilogue operands late
#ifndef RVZ_T12_KNOBS
#define RVZ_T12_KNOBS 0
#endif
using T12K = std::conditional_t<RVZ_T12_KNOBS == 1, H2Knobs<true, 1, 1, true>,
                                std::conditional_t<RVZ_T12_KNOBS == 2, H2Knobs<true, 0, 2, true>,
                                                   H2Diet>>;
constexpr int T12_TW = 4;                   // waves per team
constexpr int T12_NSLOT = RVZ_T12_SLOTS;    // task slots of the search team
constexpr int T12_SG = T12_NSLOT > 2 ? 6 : 8;   // games per slot at most (LDS: the heads rows)
constexpr int T12_RING = 32;    // LDS row ring: >= NSLOT * SG (a slot posts its rows once per cycle)
static_assert(T12_RING >= T12_NSLOT * T12_SG, "ring holds every outstanding row");

#ifndef RVZ_T12_SLEEP
#define RVZ_T12_SLEEP 1      // team-barrier polling: s_sleep between reads (0: spin)
#endif
// A 4-wave barrier on an LDS counter: each wave adds 1 once its earlier memory operations are
// released (workgroup scope, as __syncthreads' fences), then waits until the counter reaches four
// times the number of barriers it has passed.
struct TeamBar {
    unsigned* ctr;
    mutable unsigned target;
    __device__ explicit TeamBar(unsigned* c) : ctr(c), target(0) {}
    __device__ __forceinline__ void operator()() const {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        target += T12_TW;
#ifdef RVZ_PLAY_TIMING
        const unsigned long long tb0 = __builtin_amdgcn_s_memtime();
#endif
        if ((threadIdx.x & 63) == 0)
            __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        unsigned spins = 0;
        while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < target) {
            if (RVZ_T12_SLEEP) __builtin_amdgcn_s_sleep(1);
            if (++spins > (1u << 24)) {   // a team member is gone: report, and do not hang
                if ((threadIdx.x & 63) == 0) atomicOr(play_ctx().v.err, ERR_SCHED);
                break;
            }
        }
#ifdef RVZ_PLAY_TIMING   // [10]: the trunk teams' wave 0 time inside team barriers
        if ((threadIdx.x & 255) == 0 && threadIdx.x < 512 && blockIdx.x < 16384)
            atomicAdd(&g_play_t[blockIdx.x][10], __builtin_amdgcn_s_memtime() - tb0);
#endif
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
};

// head-conv rows of a trunk pass into the FC heads' LDS input of the rows' slots: board b of the
// pass is row meta[b] & 63 of slot meta[b] >> 6 (meta < 0: no board)
template <int BS>
struct HeadsSlots12 {
    float* hin;        // [NSLOT][SG][ROW]
    int meta[2];
    __device__ void store(int b, int i, float v) const {
        constexpr int CELLS = BS * BS, PIN = 2 * CELLS, PK = (PIN + 15) / 16 * 16;
        constexpr int ROW = heads_in_floats(BS) / 16;
        const int m = meta[b];
        if (m >= 0)
            hin[((m >> 6) * T12_SG + (m & 63)) * ROW + (i < PIN ? i : PK + (i - PIN))] = v;
    }
};

template <int F, int NBOARD, int CTW, int PTW, int BS>
__global__ __launch_bounds__(768) __attribute__((amdgpu_waves_per_eu(3, 3)))
void k_play12(PlayCtx ctx0) {
    (void)ctx0;   // read through play_ctx()
    using WT = WaveTilesH<F, CTW, PTW>;
    constexpr bool ILV = RVZ_H2_ILV && NBOARD == 2 && BS == 8 && PTW == 4 && WT::CG == 2;
    using GH = GeoH<NBOARD, BS, 64 * CTW * H2_TM / F, ILV>;
    using C = CfgH<F, GH::NPIX>;
    constexpr int NPOL = Geo<BS>::NPOL;
    constexpr int NS = T12_NSLOT, SG = T12_SG, R = T12_RING;
    constexpr int HROW = heads_in_floats(BS) / 16;
    static_assert(NBOARD == 2 && play_heads_lds<F, BS>(), "k_play12: the C2 geometry");
    __shared__ __attribute__((aligned(16))) char smem[2][C::BYTES];     // trunk teams' images
    __shared__ __attribute__((aligned(16))) float hin[NS * SG * HROW];   // FC heads rows
    __shared__ double spv[T12_TW][NPOL + 7];      // act scratch of the search waves
    __shared__ uint32_t key[624];                  // reset scratch (one reset at a time: rkey)
    __shared__ uint64_t ring_bits[R][3];
    __shared__ int ring_meta[R];                   // slot << 6 | row index in the slot
    __shared__ uint64_t tbits[2][NBOARD * 3];      // a trunk team's pass: (P, O, V) per board
    __shared__ int tmeta[2][NBOARD];
    __shared__ int tcnt[2];
    __shared__ unsigned bar_ctr[3];
    __shared__ unsigned ring_head, ring_claim, rkey;
    __shared__ unsigned slot_done[NS];
    __shared__ int s_exit, s_flush;
    __shared__ int st_k[NS][SG], st_f[NS][SG], st_p[NS][SG];
    __shared__ uint64_t st_bits[NS][SG * 3];
    __shared__ int q_rows[NS][SG + 16];
    __shared__ int sl_state[NS], sl_gi[NS], sl_ply[NS], sl_g0[NS], sl_ng[NS], sl_nq[NS];
    __shared__ float vpart[4][16];
    __shared__ int s_cmd[2];
    __shared__ unsigned s_tgen;
    enum : int { SL_IDLE = 0, SL_WAIT = 1, SL_SEARCH = 2, SL_EVAL = 3 };
    enum : int { CMD_EXIT = 0, CMD_SEARCH = 1, CMD_HEADS = 2, CMD_INIT = 3 };

    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int team = wave >> 2, tw = wave & 3, tt = tid & 255;
    if (tid == 0) {
        const PlayArgs& a = play_ctx().a;
        s_tgen = a.tab ? __hip_atomic_load(a.tgen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
        bar_ctr[0] = bar_ctr[1] = bar_ctr[2] = 0;
        ring_head = ring_claim = 0;
        rkey = 0;
        s_exit = 0;
        s_flush = 0;
        for (int s = 0; s < NS; ++s) {
            slot_done[s] = 0;
            sl_state[s] = SL_IDLE;
        }
    }
    __syncthreads();   // the only workgroup barrier: the teams never meet again
    bool ovf = false;
    // RVZ_PLAY_TIMING (tools/exp_play12.py TIMING=1): per workgroup shader clocks, [0]/[2] trunk
    // team 0/1 waiting for rows, [1]/[3] their passes, [4] passes, [5] single-row passes, [6] the
    // search team's search phases, [7] its heads phases, [8] its idle waits, [9] rows, [11] total
#ifdef RVZ_PLAY_TIMING
#define T12_ADD(i, v) if ((tid & 255) == 0 && blockIdx.x < 16384) atomicAdd(&g_play_t[blockIdx.x][i], (unsigned long long)(v))
#else
#define T12_ADD(i, v)
#endif
    PT_NOW(t12_start);
    if (team < 2) {
        // ---------------------------------------------------------------- a trunk team
        TeamBar tb(&bar_ctr[team]);
        for (;;) {
            PT_NOW(tw0);
            if (tt == 0) {
                const PlayArgs& a = play_ctx().a;
                int n = 0;
                unsigned k = 0, spins = 0;
                for (;;) {
                    const unsigned h = __hip_atomic_load(&ring_head, __ATOMIC_ACQUIRE,
                                                         __HIP_MEMORY_SCOPE_WORKGROUP);
                    const unsigned c = __hip_atomic_load(&ring_claim, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_WORKGROUP);
                    const unsigned avail = h - c;
                    const int flush = __hip_atomic_load(&s_flush, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_WORKGROUP);
                    const int want = avail >= 2u ? 2 : ((avail == 1u && flush) ? 1 : 0);
                    if (want > 0) {
                        unsigned exp = c;
                        if (__hip_atomic_compare_exchange_strong(
                                &ring_claim, &exp, c + (unsigned)want, __ATOMIC_RELAXED,
                                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
                            k = c;
                            n = want;
                            break;
                        }
                        continue;
                    }
                    if ((avail == 0u && __hip_atomic_load(&s_exit, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_WORKGROUP)) ||
                        (__hip_atomic_load(play_ctx().v.err, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT) & ERR_SCHED)) {
                        n = -1;
                        break;
                    }
                    if (++spins > a.spin_limit) {   // the search team stopped feeding: give up
                        atomicOr(play_ctx().v.err, ERR_SCHED);
                        __hip_atomic_store(&s_exit, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        n = -1;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
                for (int b = 0; b < NBOARD; ++b) {
                    const bool on = b < n;
                    const unsigned e = (k + (unsigned)b) % R;
                    for (int ch = 0; ch < 3; ++ch) tbits[team][3 * b + ch] = on ? ring_bits[e][ch] : 0ull;
                    tmeta[team][b] = on ? ring_meta[e] : -1;
                }
                tcnt[team] = n;
            }
            tb();
            const int n = __builtin_amdgcn_readfirstlane(tcnt[team]);
            PT_NOW(tw1);
            T12_ADD(2 * team, tw1 - tw0);
            if (n < 0) break;
            {
                const PlayArgs& a = play_ctx().a;
                HeadsSlots12<BS> hout{hin, {tmeta[team][0], tmeta[team][1]}};
                int gb[NBOARD];
#pragma unroll
                for (int b = 0; b < NBOARD; ++b) gb[b] = -1;   // bitboard stem: no planes read
                const int t = opaque_tid() & 255;
                h2_pass<F, NBOARD, CTW, PTW, BS, HeadsSlots12<BS>, T12K, TeamBar>(
                    smem[team], a.x, gb, tbits[team], a.prm, a.L, a.blob, a.n_blocks, hout, t,
                    t & 63, __builtin_amdgcn_readfirstlane((t >> 6) & 3), ovf, tb);
            }
            tb();   // every head-conv row of the pass is in hin
            PT_NOW(tw2);
            T12_ADD(2 * team + 1, tw2 - tw1);
            T12_ADD(4, 1);
            T12_ADD(5, n == 1 ? 1 : 0);
            if (tt == 0) {
                for (int b = 0; b < n; ++b)
                    __hip_atomic_fetch_add(&slot_done[tmeta[team][b] >> 6], 1u, __ATOMIC_RELEASE,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
    } else {
        // ---------------------------------------------------------------- the search team
        TeamBar sb(&bar_ctr[2]);
        int E, G, gpw, total;
        {
            const PlayCtx& c = play_ctx();
            E = c.v.E;
            G = c.v.G;
            gpw = c.a.gpw;
            total = c.a.n_groups * c.a.plies;
        }
        int n_rows = 0;
        unsigned n_hits = 0, n_ins = 0;
        double* sp = spv[tw];
        bool drained = false;    // the queue has no task left
        unsigned idle = 0;
        for (;;) {
            PT_NOW(ts0);
            // the leader picks the next step: a slot's heads (its rows are all evaluated), a
            // slot's search phase, a slot's start (its task's previous ply is published), or a
            // new task for an idle slot; with nothing to do it lets the trunk teams take a single
            // row (s_flush) and waits
            if (tt == 0) {
                const PlayCtx& c = play_ctx();
                const PlayArgs& a = c.a;
                int cmd = -1, slot = -1;
                for (;;) {
                    for (int s = 0; s < NS && cmd < 0; ++s) {
                        const int st = sl_state[s];
                        if (st == SL_EVAL &&
                            __hip_atomic_load(&slot_done[s], __ATOMIC_ACQUIRE,
                                              __HIP_MEMORY_SCOPE_WORKGROUP) == (unsigned)sl_nq[s]) {
                            cmd = CMD_HEADS;
                            slot = s;
                        } else if (st == SL_SEARCH) {
                            cmd = CMD_SEARCH;
                            slot = s;
                        } else if (st == SL_WAIT &&
                                   (int)__hip_atomic_load(a.q_done + sl_gi[s], __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT) >= sl_ply[s]) {
                            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                            cmd = CMD_INIT;
                            slot = s;
                        } else if (st == SL_IDLE && !drained) {
                            const bool failed = __hip_atomic_load(c.v.err, __ATOMIC_RELAXED,
                                                                  __HIP_MEMORY_SCOPE_AGENT) &
                                                ERR_SCHED;
                            const unsigned t =
                                failed ? (unsigned)total
                                       : __hip_atomic_fetch_add(a.q_next, 1u, __ATOMIC_RELAXED,
                                                                __HIP_MEMORY_SCOPE_AGENT);
                            if ((int)t >= total) {
                                drained = true;
                            } else {
                                const int gi = (int)(t % (unsigned)a.n_groups);
                                sl_gi[s] = gi;
                                sl_ply[s] = (int)(t / (unsigned)a.n_groups);
                                sl_g0[s] = gi * gpw;
                                sl_ng[s] = min(gpw, G - gi * gpw);
                                sl_state[s] = SL_WAIT;
                                idle = 0;
                            }
                        }
                    }
                    if (cmd >= 0) break;
                    bool busy = !drained;
                    for (int s = 0; s < NS; ++s) busy |= sl_state[s] != SL_IDLE;
                    if (!busy) {
                        cmd = CMD_EXIT;
                        break;
                    }
                    __hip_atomic_store(&s_flush, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (++idle > a.spin_limit ||
                        (__hip_atomic_load(c.v.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) &
                         ERR_SCHED)) {
                        atomicOr(c.v.err, ERR_SCHED);
                        cmd = CMD_EXIT;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
                if (cmd != CMD_EXIT)
                    __hip_atomic_store(&s_flush, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                idle = cmd == CMD_EXIT ? idle : 0;
                s_cmd[0] = cmd;
                s_cmd[1] = slot;
            }
            sb();
            const int cmd = __builtin_amdgcn_readfirstlane(s_cmd[0]);
            const int s = __builtin_amdgcn_readfirstlane(s_cmd[1]);
            PT_NOW(ts1);
            T12_ADD(8, ts1 - ts0);
            if (cmd == CMD_EXIT) break;
            const int g0 = __builtin_amdgcn_readfirstlane(sl_g0[s]);
            const int ng = __builtin_amdgcn_readfirstlane(sl_ng[s]);
            const int ply0 = __builtin_amdgcn_readfirstlane(sl_ply[s]);
            if (cmd == CMD_INIT) {   // a game whose ply budget this task's ply reaches starts done
                const int32_t* bud = play_ctx().a.budget;
                for (int j = tt; j < ng; j += 256) {
                    st_k[s][j] = 0;
                    st_f[s][j] = (bud && ply0 >= bud[g0 + j]) ? PF_DONE : 0;
                    st_p[s][j] = 0;
                }
                if (tt == 0) sl_state[s] = SL_SEARCH;
                sb();
                continue;
            }
            if (cmd == CMD_SEARCH) {
                // each game not waiting for its row advances until it queues the next row or has
                // committed its ply (k_play's search phase, one slot)
                for (int j = tw; j < ng; j += T12_TW) {
                    const PlayCtx& c = play_ctx();
                    const View& v = c.v;
                    const PlayArgs& a = c.a;
                    const int lane = opaque_tid() & 63;
                    const int g = g0 + j;
                    int f = __builtin_amdgcn_readfirstlane(st_f[s][j]);
                    if (f & (PF_QUEUED | PF_DONE)) continue;
                    int k = __builtin_amdgcn_readfirstlane(st_k[s][j]);
                    int np = __builtin_amdgcn_readfirstlane(st_p[s][j]);
                    for (;;) {
                        unsigned long long ab = 0;
                        if (k < E) {
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
                                const ExpIn x = expand_load<BS>(v, g, lane, a.logits, a.value);
                                const int rn =
                                    expand_backup_phase<BS>(v, g, lane, x, 1, &root_meta, ab);
                                if (rn >= 0) root_n = rn;
                                f &= ~PF_READY;
                            }
                            const int bsz = min(a.B, a.S - k * a.B);
                            const int copies = select_phase<BS, float>(
                                v, g, lane, first, bsz, k, root, root_meta, root_n, carry, a.x,
                                a.need, ab, st_bits[s] + 3 * j);
                            ++k;
                            if (copies > 0 && !(k == E && a.skip_last)) {
                                if (a.tab) {
                                    const uint64_t P = st_bits[s][3 * j], O = st_bits[s][3 * j + 1],
                                                   Vb = st_bits[s][3 * j + 2];
                                    if (__popcll(P | O) <= a.tmaxd &&
                                        tab_lookup<BS>(a, s_tgen, P, O, Vb, lane, g)) {
                                        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
                                        f |= PF_READY;
                                        ++n_hits;
                                        continue;
                                    }
                                }
                                f |= PF_QUEUED;
                                break;
                            }
                            continue;
                        }
                        bool over = false;
                        double* outp = a.out_p;
                        if (a.rec_black) {
                            const size_t ri = (size_t)(ply0 + np) * v.G + g;
                            if (lane == 0) {
                                a.rec_black[ri] = v.black[g];
                                a.rec_white[ri] = v.white[g];
                                a.rec_side[ri] = v.status[(size_t)g * 4];
                            }
                            outp = a.rec_p + (size_t)(ply0 + np) * v.G * Geo<BS>::NPOL;
                        }
                        const int idx = act_game<BS>(v, g, lane, sp, (f & PF_READY) ? 1 : 2,
                                                     a.logits, 1, a.value, a.temperature, nullptr,
                                                     1, a.out_idx, outp, &over);
                        f &= ~PF_READY;
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
                            // the reset scratch is one LDS key: one search wave at a time
                            sd = __shfl(sd, 0);
                            if (lane == 0) {
                                while (__hip_atomic_exchange(&rkey, 1u, __ATOMIC_ACQUIRE,
                                                             __HIP_MEMORY_SCOPE_WORKGROUP) != 0u)
                                    __builtin_amdgcn_s_sleep(1);
                            }
                            __builtin_amdgcn_wave_barrier();
                            reset_game<BS>(v, g, lane, (uint32_t)(sd & 0xFFFFFFFFll), key);
                            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
                            if (lane == 0)
                                __hip_atomic_store(&rkey, 0u, __ATOMIC_RELEASE,
                                                   __HIP_MEMORY_SCOPE_WORKGROUP);
                        }
                        ++np;
                        k = 0;
                        f |= PF_DONE;   // a task is one ply
                        break;
                    }
                    if (lane == 0) {
                        st_k[s][j] = k;
                        st_f[s][j] = f;
                        st_p[s][j] = np;
                    }
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // a publish may follow
                sb();
                if (tt == 0) {   // the queued rows, in game order, to the ring
                    int n = 0;
                    const unsigned h = ring_head;
                    for (int j = 0; j < ng; ++j) {
                        const int fj = st_f[s][j];
                        if (!(fj & PF_QUEUED)) continue;
                        st_f[s][j] = fj | PF_EVAL;
                        const unsigned e = (h + (unsigned)n) % R;
                        for (int ch = 0; ch < 3; ++ch) ring_bits[e][ch] = st_bits[s][3 * j + ch];
                        ring_meta[e] = (s << 6) | n;
                        q_rows[s][n++] = g0 + j;
                    }
                    for (int i = n; i < n + 16; ++i) q_rows[s][i] = -1;
                    sl_nq[s] = n;
                    n_rows += n;
                    if (n > 0) {
                        sl_state[s] = SL_EVAL;
                        __hip_atomic_store(&ring_head, h + (unsigned)n, __ATOMIC_RELEASE,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
                    } else {   // every game committed its ply: publish the group's ply
                        const PlayArgs& a = play_ctx().a;
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        __hip_atomic_store(a.q_done + sl_gi[s], (unsigned)(ply0 + 1),
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        sl_state[s] = SL_IDLE;
                    }
                }
                sb();
                {
                    PT_NOW(ts2);
                    T12_ADD(6, ts2 - ts1);
                }
                continue;
            }
            // CMD_HEADS: the slot's rows are all evaluated: FC heads, table inserts, flags
            const int nq = __builtin_amdgcn_readfirstlane(sl_nq[s]);
            {
                const PlayArgs& a = play_ctx().a;
                heads_fc16<BS, HeadRowsList, true, false, SG, TeamBar>(
                    a.work, HeadRowsList{q_rows[s]}, a.prm, a.L, a.logits, a.value,
                    hin + s * SG * HROW, vpart, opaque_tid() & 255, sb);
            }
            if (play_ctx().a.tab) {   // the heads ended with a team barrier: the rows are written
                for (int i = tw; i < nq; i += T12_TW) {
                    const PlayArgs& a = play_ctx().a;
                    const int j = q_rows[s][i] - g0;
                    const uint64_t P = st_bits[s][3 * j], O = st_bits[s][3 * j + 1],
                                   Vb = st_bits[s][3 * j + 2];
                    if (__popcll(P | O) <= a.tmaxd)
                        n_ins += tab_insert<BS>(a, s_tgen, P, O, Vb, opaque_tid() & 63, q_rows[s][i]);
                }
            }
            if (tt == 0) {
                for (int j = 0; j < ng; ++j) {
                    const int fj = st_f[s][j];
                    if (fj & PF_EVAL) st_f[s][j] = (fj & ~(PF_QUEUED | PF_EVAL)) | PF_READY;
                }
                slot_done[s] = 0;
                sl_state[s] = SL_SEARCH;
            }
            sb();
            {
                PT_NOW(ts3);
                T12_ADD(7, ts3 - ts1);
            }
        }
        __hip_atomic_store(&s_exit, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        T12_ADD(9, n_rows);
        {
            PT_NOW(t12_end);
            T12_ADD(11, t12_end - t12_start);
        }
        unsigned long long* rows = play_ctx().a.rows;
        if (rows && tt == 0) atomicAdd(rows, (unsigned long long)n_rows);
        unsigned long long* ts = play_ctx().a.tstats;
        if (ts && (tt & 63) == 0) {
            if (n_hits) atomicAdd(ts, (unsigned long long)n_hits);
            if (n_ins) atomicAdd(ts + 1, (unsigned long long)n_ins);
        }
    }
    float* ovw = play_ctx().a.ovf;
    if (ovf && ovw) *ovw = 1.0f;   // benign race: every writer stores 1
}
