/*
 * rvz.h — C-ABI of the MI355X-native Reversi self-play engine (librvz.so, gfx950).
 *
 * The reference (RandomMike1280/AlphaZero-Reversi) has no FFI on this path: its boundary is three
 * duck-typed Python protocols (game / model / MCTS). Each entry point below replaces one piece of
 * that surface; the line each one replaces is cited next to it. The Python host mirror in
 * alphazero-reversi_amd/rvz (ReversiGame, MCTS, SelfPlay) binds these with ctypes
 * (INTEGRATION.md shows the binding a reference maintainer would add).
 *
 * Conventions
 *  - Every array argument is a DEVICE pointer (HBM, e.g. torch.Tensor.data_ptr()) unless the
 *    comment says "host". Work is enqueued on the engine's stream (rvz_set_stream) or on the
 *    stream argument; nothing here synchronises except rvz_sync / rvz_check.
 *  - Squares are row-major: square s <-> (row, col) = (s / S, s % S), bit s of a bitboard
 *    (board.py:49). The policy index S*S is the pass move (-1, -1) (mcts.py:666-667,687-688).
 *  - Game status is int32[4] per game: {side to move 1|2, game_over 0|1, winner -1 (None)|0|1|2,
 *    passed_moves_in_a_row} (board.py:33-37, game.py:20-23).
 *  - Return codes: RVZ_OK (0) or a negative RVZ_E*; rvz_last_error() explains the last failure.
 *    Game-level illegality is data, not an error: make_move's False is written to out_ok.
 *  - One engine per device per process; not re-entrant. The caller owns every in/out buffer.
 */
#ifndef RVZ_H
#define RVZ_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RVZ_OK 0
#define RVZ_DONE 1          /* rvz_search_step: every batch of this search has been issued */
#define RVZ_EINVAL (-22)
#define RVZ_ENOMEM (-12)
#define RVZ_EHIP (-5)
#define RVZ_EDEVICE (-71)   /* a kernel raised its device-side error word (rvz_check) */

#define RVZ_LEAF_F32 0      /* leaf planes in float32, exactly game.get_canonical_state() */
#define RVZ_LEAF_BF16 1     /* the same 0/1 planes as bfloat16 (exact) for a bf16 evaluator */

/* Live-row counts of a compacted leaf batch (rvz_search_compact, the n_live argument of
 * rvz_resnet_*_ex): the rows are handed out per stripe of RVZ_LIVE_STRIPE rows (game g draws
 * from stripe g / RVZ_LIVE_STRIPE), one int32 counter per stripe, RVZ_LIVE_PITCH int32 apart;
 * stripe s has its live rows at [s * RVZ_LIVE_STRIPE, s * RVZ_LIVE_STRIPE + n_live[s * PITCH]). */
#define RVZ_LIVE_STRIPE 128
#define RVZ_LIVE_PITCH 16

typedef struct rvz_engine rvz_engine;

typedef struct rvz_config {
    int32_t board_size;       /* 8 (reference; board.py:27-28) or 6 (build-defined variant) */
    int32_t n_games;          /* games owned by this engine (one tree each) */
    int32_t num_simulations;  /* MCTS(num_simulations=800)  mcts.py:197 */
    int32_t batch_size;       /* MCTS(batch_size=64)        mcts.py:198; ceil(sims/batch) <= 64 */
    double c_puct;            /* MCTS(c_puct=1.0)           mcts.py:197 */
    int32_t device;           /* HIP device ordinal */
    int32_t leaf_dtype;       /* RVZ_LEAF_F32 | RVZ_LEAF_BF16 */
} rvz_config;

/* ---- lifetime -------------------------------------------------------------------------- */
/* replaces MCTS.__init__ (mcts.py:197-235) + the per-game ReversiGame() of self_play.py:71 */
int rvz_create(const rvz_config *cfg /* host */, rvz_engine **out /* host */);
void rvz_destroy(rvz_engine *e);
const char *rvz_last_error(const rvz_engine *e);          /* e may be NULL: last create error */
int rvz_set_stream(rvz_engine *e, void *hip_stream);        /* hipStream_t; NULL = default */
int rvz_sync(rvz_engine *e);                                /* hipStreamSynchronize */
int rvz_check(rvz_engine *e, int32_t *host_err);            /* sync + read/clear device error */
int rvz_version(void);

/* ---- env, engine-owned (board.py / game.py over n_games boards in HBM) --------------------- */
/* Reset games to the start position (board.py:25-39) and seed each game's numpy-compatible
 * MT19937 stream with seeds[g] (np.random.seed, the RNG behind mcts.py:684). mask: reset only
 * games with mask[g] != 0 (NULL = all). */
int rvz_env_reset(rvz_engine *e, const uint32_t *seeds, const uint8_t *mask);
/* The self-play loop's per-ply bookkeeping (self_play.py:80-101 with every game slot kept busy):
 * plies[g] += 1 when idx[g] >= 0 (rvz_act committed a move); with reset != 0 a game that is over
 * adds 1 to done[g], takes seeds[g] += stride (int64, in place) and restarts from the start
 * position with np.random.seed(seeds[g] mod 2^32) semantics, as rvz_env_reset. idx: rvz_act's
 * out_idx; plies, done: int64 [n_games] per-game counters (sum them to read totals). */
int rvz_env_autoreset(rvz_engine *e, const int32_t *idx, int64_t *seeds, int64_t stride,
                      int64_t *plies, int64_t *done, int32_t reset);
/* The move-sampling draws of each game (np.random.choice's one random_sample() per move,
 * mcts.py:684): rvz_env_reset fills game g's RVZ_DRAWS values from np.random.seed(seeds[g]);
 * rvz_env_set_draws replaces them with u[g][0..RVZ_DRAWS) (float64, device) and rewinds every
 * game to its first value, so a caller can hand each game its slice of ONE stream — the
 * reference's generate_games draws every game's moves in sequence from the global np.random
 * state (self_play.py:66-101, seeded once at pipeline.py:74-80). rvz_env_draws writes the number
 * of values each game has consumed since then (int32 [n_games]; rvz_act / rvz_play at
 * temperature 0 draw none). A game that would draw more than RVZ_DRAWS sets device error bit 1. */
#define RVZ_DRAWS 64
int rvz_env_set_draws(rvz_engine *e, const double *u);
int rvz_env_draws(rvz_engine *e, int32_t *out_pos);
int rvz_env_get(rvz_engine *e, uint64_t *black, uint64_t *white, int32_t *status);
int rvz_env_set(rvz_engine *e, const uint64_t *black, const uint64_t *white, const int32_t *status);
/* ReversiGame.get_valid_moves (game.py:72-79 -> board.py:70-133) as a bitmask per game */
int rvz_env_legal(rvz_engine *e, uint64_t *out_mask);
/* ReversiGame.make_move (game.py:36-70 -> board.py:135-251); sq[g] = -1 is the pass (-1,-1) */
int rvz_env_apply(rvz_engine *e, const int32_t *sq, int32_t *out_ok);

/* ---- board kernels on caller arrays (stateless; n boards) ------------------------------ */
int rvz_board_legal(int32_t board_size, int32_t n, const uint64_t *black, const uint64_t *white,
                    const int32_t *status, uint64_t *out_mask, void *hip_stream);
int rvz_board_apply(int32_t board_size, int32_t n, uint64_t *black, uint64_t *white,
                    int32_t *status, const int32_t *sq, int32_t *out_ok, void *hip_stream);
/* ReversiGame.get_canonical_state (game.py:131-162): float32 [n, 3, S, S] */
int rvz_board_canonical(int32_t board_size, int32_t n, const uint64_t *black,
                        const uint64_t *white, const int32_t *status, float *out,
                        void *hip_stream);

/* F.softmax(policy_logits, dim=1) of _process_batch (mcts.py:596) over n rows of S*S+1 logits:
 * bitwise the probabilities the expand computes when rvz_search_submit gets logits (is_logits = 1)
 * and inside rvz_play (the same device function). The tests feed the oracle with it. */
int rvz_policy_softmax(int32_t board_size, int32_t n, const float *logits, float *probs,
                       void *hip_stream);

/* ---- search (MCTS.search, mcts.py:322-407, one tree per game, lockstep over games) -------- */
/* New root per live game from the engine's env state (mcts.py:334-341). */
int rvz_search_begin(rvz_engine *e);
/* Issue the next batch (mcts.py:348-392 up to the NN call): traversals, immediate terminal
 * backups, _process_batch pass 1. Writes the leaf planes of game g into row g of leaf_x
 * ([n_games, 3, S, S], leaf_dtype) and need[g] = the number of queued traversal copies that
 * wait for row g (0: row g unused this batch). Returns RVZ_DONE (and does nothing) when the
 * search has issued all ceil(num_simulations / batch_size) batches. */
int rvz_search_step(rvz_engine *e, void *leaf_x, int32_t *need);
/* _process_batch pass 2 (mcts.py:600-623): expand every waiting leaf from policy row g and back
 * up value[g]. policy is [n_games, S*S+1] float32: softmaxed probabilities (is_logits = 0,
 * exactly mcts.py:596's input) or raw logits (is_logits = 1: softmax fused into the kernel).
 * Deferred: the work runs at the head of the next rvz_search_step / rvz_act launch (fused into
 * that kernel) or of rvz_search_visits / rvz_tree_export, so policy and value must stay valid and
 * unmodified on the stream until that call. */
int rvz_search_submit(rvz_engine *e, const float *policy, int32_t is_logits, const float *value);
/* Instead of rvz_search_submit for the LAST batch of a search (after the rvz_search_step that
 * issued it): leave its leaves unevaluated. The evaluation of the last batch feeds only state the
 * discarded tree never reads (the leaf's children priors, W along the path; mcts.py:600-640), so
 * rvz_search_visits / rvz_act then back up the visit counts alone and return exactly the visits,
 * p and move of the evaluated search (tests/test_gpu_search.py::test_skip_last_eval_bit_exact).
 * Needs a search of at least two batches (num_simulations > batch_size; RVZ_EINVAL otherwise:
 * a single batch's leaf is the root, whose expansion the act needs; rvz_play's skip_last_eval
 * is ignored for such searches).
 * Off unless called (one NN call fewer per move; not the reference's call sequence). bench.py's
 * headline uses it by default (--evals table, and --evals lazy: the memo + this, so the skipped
 * evaluation is made later only if a search reaches that position; rvz_play's skip_last_eval is
 * the same; --evals reference turns it off). */
int rvz_search_skip(rvz_engine *e);
/* Compacted leaf batches (on != 0; off by default): rvz_search_step writes the leaves that need an
 * evaluation (need[g] > 0; mcts.py:544-623 evaluates exactly those) to the first rows of their
 * game's stripe of RVZ_LIVE_STRIPE rows, in an unspecified order, and rvz_search_submit reads each
 * game's policy / value from that game's row. The per-stripe counts stay on the device:
 * rvz_search_live_count returns the address of the most recently issued batch's counts (layout
 * above; stable for the engine's life per batch index of a search, so a captured graph may bake
 * it in), for the n_live argument of rvz_resnet_*_ex. An evaluator that ignores them and
 * evaluates all n_games rows gives the same search. Visits, p and moves are identical to the
 * uncompacted search. */
int rvz_search_compact(rvz_engine *e, int32_t on);
const int32_t *rvz_search_live_count(const rvz_engine *e);
/* NN-output memo across consecutive searches (on != 0; off by default). The reference rebuilds
 * the tree at every move (mcts.py:334), so the next search's root — the child the move went to —
 * and often some of its descendants are positions this game's previous search already expanded
 * from an NN evaluation. With the memo on, such a leaf is expanded from that earlier output (the
 * priors of its children and its value, kept in the other half of the node pool) instead of
 * being queued for the evaluator: need[g] = 0 and no leaf row for it. A leaf evaluator's row
 * outputs must depend only on the position (true of rvz_resnet_fwd_h2 and any deterministic
 * per-row net), and the net must not change between the two searches: call
 * rvz_search_memo_reset after new weights. Visits, p and moves are identical to the search
 * without the memo (tests/test_gpu_memo.py); it changes only how many rows are evaluated.
 * The memo needs a second half of the node pool (the previous tree): the first call with on != 0
 * reallocates the pool (device pointers change), so enable it before capturing a graph.
 * The carried links are dropped automatically by rvz_env_reset / rvz_env_autoreset (per game),
 * rvz_env_set, rvz_env_apply, rvz_act without apply and an abandoned search. Not inside a
 * search. */
int rvz_search_memo(rvz_engine *e, int32_t on);
int rvz_search_memo_reset(rvz_engine *e);
/* Host int64: the live rows of every evaluated batch of every search completed by rvz_act since
 * compaction was first enabled (0 if never enabled; a batch left by rvz_search_skip is not
 * counted); synchronises the engine stream. */
int rvz_search_rows_total(rvz_engine *e, int64_t *out /* host */);
/* {move: child.visit_count} (mcts.py:406-407) as int32 [n_games, S*S+1] */
int rvz_search_visits(rvz_engine *e, int32_t *out);
/* get_action_probs' tail (mcts.py:656-692) + SelfPlay's make_move (self_play.py:98):
 * p (float64 [n_games, S*S+1]) and the chosen index (int32 [n_games]; S*S = pass, -2 = game
 * already over) per game. Samples with each game's MT19937 stream, or with u[g] when u != NULL
 * (float64 [n_games]; the value np.random.random_sample() would return). apply != 0 then plays
 * the move on the engine's env (ReversiGame.make_move semantics). */
int rvz_act(rvz_engine *e, double temperature, const double *u, int32_t apply, int32_t *out_idx,
            double *out_p);

/* ---- fused self-play ---------------------------------------------------------------------
 * Replaces SelfPlay.generate_games' ply loop (self_play.py:80-101: MCTS.search + get_action_probs
 * + make_move, mcts.py:322-407 and :642-694) together with its leaf evaluator
 * (AlphaZeroNetwork.predict, network.py:136-158) when the evaluator is the h2 ResNet: ONE launch in
 * which each workgroup plays its own games, every game committing `plies` plies (each a full
 * search of num_simulations), with the per-ply bookkeeping of rvz_env_autoreset. The games, moves,
 * p and counters are bit-identical to the pull-style loop (rvz_search_step / the
 * rvz_resnet_fwd_h2 evaluator with logits / rvz_search_submit / rvz_act / rvz_env_autoreset) on
 * the same engine state; the engine's memo setting applies; compaction is inherent (only the live
 * leaves are evaluated). Not inside a search; graph-capturable (no allocation, no sync). */
typedef struct rvz_play_args {
    const float *params;         /* packed fp32 net (rvz_resnet_params_size layout) */
    const uint16_t *blob;        /* its h2 weight blob (rvz_resnet_h2_weights), 16-byte aligned */
    int32_t filters;             /* 64 | 128 (| 256 on board 8) */
    int32_t blocks;              /* residual blocks */
    float *scratch;              /* rvz_play_scratch_size(e) floats, 16-byte aligned */
    float *ovf;                  /* the evaluator's sticky f16-overflow word (set to 1), nullable */
    int32_t plies;               /* plies every game commits in this call, >= 1 */
    int32_t skip_last_eval;      /* each search's last batch unevaluated (rvz_search_skip) */
    int32_t reset;               /* finished games restart (rvz_env_autoreset's reset) */
    int32_t games_per_workgroup; /* > 0: static schedule, each workgroup owns that many games for
                                    every ply; <= 0: task queue, the workgroups draw (group of
                                    -games_per_workgroup games, ply) tasks (0: 4 games) */
    double temperature;
    int64_t *seeds;              /* int64 [n_games], as rvz_env_autoreset */
    int64_t seed_stride;
    int64_t *plies_done;         /* int64 [n_games], += 1 per committed move */
    int64_t *games_done;         /* int64 [n_games], += 1 per finished game (reset != 0) */
    int32_t *out_idx;            /* int32 [n_games]: each game's last act (as rvz_act) */
    double *out_p;               /* float64 [n_games, S*S+1]: its policy vector */
    int32_t *hist;               /* int32 [plies][n_games]: every act's index, nullable */
    int64_t *rows_evaluated;     /* int64 [1] += the leaf rows evaluated by the call, nullable */
    const int32_t *ply_budget;   /* int32 [n_games]: game g commits min(plies, ply_budget[g])
                                    plies in this call (<= 0: none; it is left as it is), nullable
                                    (every game commits `plies`). bench.py staggers the games'
                                    phases with it (game g at ply g mod 60 of its game) */
    int64_t *table_stats;        /* int64 [2] += {table hits, table inserts} (rvz_play_table), nullable */
    /* Self-play records (self_play.py:88-101, the trainer's input; all four or none): for every
     * act of the call, at [p][g] with p = the act's ply within the call, the position before the
     * move (board bitboards and the side to move) and get_action_probs' vector (rec_p float64
     * [plies][n_games][S*S+1]); hist holds the move. out_p is then not written. */
    uint64_t *rec_black;         /* uint64 [plies][n_games], nullable */
    uint64_t *rec_white;
    int32_t *rec_side;           /* int32 [plies][n_games] */
    double *rec_p;
} rvz_play_args;
/* A task-queue wait that times out (a workgroup waiting for its group's previous ply, bounded
 * spin) sets device error bit 16 (rvz_check): the other workgroups then stop drawing tasks and the
 * launch drains, leaving games at different ply counts. The engine state is then undefined until
 * every game is reset (rvz_env_reset). */
int64_t rvz_play_scratch_size(const rvz_engine *e);
int rvz_play(rvz_engine *e, const rvz_play_args *a);
/* Cross-game NN-output table for rvz_play (off by default; slots = 0 turns it off and frees it).
 * The reference evaluates every leaf (mcts.py:544-623) and carries an inert transposition table
 * for reuse (mcts.py:228-320, 368-385); here, a leaf whose position (mover, opponent, legal-move
 * bitboards: exactly the NN input planes, game.py:131-162) has at most max_discs discs is looked
 * up in a device hash table of `slots` entries (a power of two) before it is queued, and an
 * evaluated row of such a position is stored: a hit expands the leaf from the stored logits and
 * value, which are bitwise what the h2 evaluator returns for that position (its row outputs depend
 * only on the row: tests/test_gpu_network.py), from any earlier evaluation by any game of the
 * engine. Visits, p and moves are identical with and without it (tests/test_gpu_table.py); it
 * changes how many rows are evaluated. Like the memo it requires unchanged weights:
 * rvz_search_memo_reset (new weights in place) starts a new table generation, and so does a call
 * of rvz_play with another weight blob (a kernel on the stream: refused with RVZ_EINVAL while the
 * stream is capturing, so a captured graph never replays it; play once eagerly per evaluator
 * before capturing). 8-byte {datum, generation} granules written and read with agent-scope
 * accesses, so workgroups on every XCD share it without fences. Not inside a search. */
int rvz_play_table(rvz_engine *e, int64_t slots, int32_t max_discs);
/* The per-XCD pass gate of rvz_play's 8x8 forms of 128 and 256 filters (the task-queue schedule).
 * There every trunk pass streams the whole f16-pair weight set (10x128: 11.8 MB), which the
 * workgroups of an XCD, each at its own layer, cannot share through the XCD's 4 MB L2. With the
 * gate a workgroup about to start a pass waits until `fraction` of its XCD's running workgroups
 * have arrived or `timeout_us` has passed since its own arrival, so the XCD's passes start
 * together and read each layer's weights together; a workgroup arriving within `late_us` of the
 * latest round's opening joins that round at once. Timing only: games, moves and counters are
 * identical with any setting (tests/test_gpu_play.py). fraction 0 turns it off; fraction < 0
 * restores the default (0.8, 400 us, 200 us: C3 +8-10% on MI355X, C3's workload at 10x256
 * +10%). The environment
 * variable RVZ_PLAY_GATE="fraction,us[,late_us]" overrides the setting (experiments). */
int rvz_play_gate(rvz_engine *e, double fraction, double timeout_us, double late_us);

/* ---- introspection (tests / bench) -------------------------------------------------------- */
/* Stream-ordered HIP event timer, events without system fence (the engine's own launch timing
 * uses the same): record i / j around launches on a stream, rvz_timer_elapsed synchronises on j
 * and returns the ms between them (host float). Not for stream capture. */
typedef struct rvz_timer rvz_timer;
int rvz_timer_create(int32_t n_events, rvz_timer **out);
int rvz_timer_record(rvz_timer *t, int32_t i, void *hip_stream);
int rvz_timer_elapsed(rvz_timer *t, int32_t i, int32_t j, float *ms /* host */);
void rvz_timer_destroy(rvz_timer *t);

/* Host copy of per-engine counters: [0] search batches issued, [1] kernel launches. */
int rvz_counters(const rvz_engine *e, int64_t *out2 /* host */);
/* Algorithmic-byte counters (bench roofline): while enabled, every search kernel adds the bytes
 * its algorithm must move (nodes scanned, planes/rows written, backups) to a device counter;
 * read returns host int64[3] = {k_step (expand + select), k_act (expand + act), standalone
 * k_expand_backup} since the last enable. Off by default (one atomic per game per launch). */
int rvz_stats_enable(rvz_engine *e, int32_t on);
int rvz_stats_read(rvz_engine *e, int64_t *out3 /* host */);
/* Launch timing (bench roofline): while enabled, every k_step (rvz_search_step) and k_act
 * (rvz_act) launch is bracketed by a pair of HIP events recorded on the engine stream, created with
 * hipEventDisableSystemFence (no cache write-back/invalidate around the timed kernel). read
 * synchronises and returns the mean milliseconds and the launch counts {k_step, k_act}. */
int rvz_timing_enable(rvz_engine *e, int32_t on);
int rvz_timing_read(rvz_engine *e, double *out_ms /* host [2] */, int32_t *out_n /* host [2] */);
/* Tree export for tests: nodes_out [n_games * nodes_per_game] x {int32 N, f32 W, f32 P, f32 C},
 * meta_out [n_games * nodes_per_game] uint32 (device). nodes_per_game = rvz_tree_nodes(). */
int rvz_tree_nodes(const rvz_engine *e);
int rvz_tree_export(rvz_engine *e, void *nodes_out, uint32_t *meta_out);
/* Sizes of the engine's device-resident state, for DESIGN/bench accounting (host out). */
int rvz_footprint(const rvz_engine *e, int64_t *bytes_tree, int64_t *bytes_env);

/* ---- the leaf evaluator (the policy/value net, the boundary's callee) ---- */
/* The reference's AlphaZeroNetwork forward (network.py:30-117, BN folded): x float32
 * [n, 3, board, board] (the leaf planes) -> logits float32 [n, board^2 + 1], value float32 [n].
 * params: the packed fp32 buffer laid out as in csrc/rvz_resnet_common.hip.h
 * (rvz.network.pack_resnet_params), 16-byte aligned, of rvz_resnet_params_size(board, filters,
 * blocks) floats (negative: unsupported shape). filters 64 or 128 (boards 8 and 6) or 256 (board
 * 8; the fused rvz_play too), any block count.
 * work: float scratch of rvz_resnet_work_size(n) elements (the 1x1-conv head outputs handed from
 * the trunk launch to the FC-heads launch, + the overflow word). */
int64_t rvz_resnet_params_size(int32_t board, int32_t filters, int32_t blocks);
int64_t rvz_resnet_work_size(int32_t n);
/* The batched FC heads alone (work -> logits, value; f32 MFMA, fp32 products and sums). */
int rvz_resnet_heads_fc(int32_t board, const float *work, int32_t n, const float *params,
                        int32_t filters, int32_t blocks, float *logits, float *value,
                        void *hip_stream);

/* The forward, fp32 emulated on the f16 MFMA with two parts per operand (the leaf evaluator):
 * x = x0 + x1 (f16 each, 22 significant bits), weights pre-scaled per output channel by a power
 * of two, the three partial products x0w0 + x0w1 + x1w0 accumulated in one fp32
 * accumulator (error of an fp32 GEMM; see csrc/rvz_resnet.hip k_resnet_h2). Boards 8 and 6.
 * blob: rvz_resnet_h2_weights' output (scaled f16 parts + inverse scales, then a range table of
 * {max over output channels of sum |w|, max |bias|} per conv layer, once per parameter update),
 * rvz_resnet_h2_size(filters, blocks) uint16 elements, 16-byte aligned.
 * Activation range: a pass whose unscaled activations reach f16's limit (65520) re-runs the
 * boards that did with their images scaled by a power of two chosen from the range table's
 * bounds (exact; fp32-class relative to the board's largest activation); other boards' outputs
 * are unchanged bit for bit.
 * work: rvz_resnet_work_size(n) floats (16-byte aligned); work[n * 192] (zero it before the first
 * use) is set to 1 (never cleared by the kernel) if a scaled re-run still overflowed (a bound
 * error: the outputs are not valid; no finite net reaches it); words n * 192 + 2, 3 hold the trunk's 64-bit board-unit
 * counter (units dealt to workgroups in start order; any initial value below 2^63). A misaligned
 * work returns RVZ_EINVAL. A workspace must not be shared by launches that can run concurrently
 * (two streams, or one buffer reused across overlapping launches): every launch claims its
 * board units from the counter, and interleaved claims would skip or repeat units silently.
 * Give each stream (each lane) its own workspace. */
int64_t rvz_resnet_h2_size(int32_t filters, int32_t blocks);
int rvz_resnet_h2_weights(const float *params, int32_t filters, int32_t blocks, uint16_t *blob,
                          void *hip_stream);
int rvz_resnet_fwd_h2(int32_t board, const float *x, int32_t n, const float *params,
                      const uint16_t *blob, int32_t filters, int32_t blocks, float *work,
                      float *logits, float *value, void *hip_stream);
int rvz_resnet_trunk_h2(int32_t board, const float *x, int32_t n, const float *params,
                        const uint16_t *blob, int32_t filters, int32_t blocks, float *work,
                        void *hip_stream);
/* Extended forms. n_live (device int32 per-stripe counts as laid out at RVZ_LIVE_STRIPE, nullable):
 * only the live rows of each stripe are evaluated (a compacted leaf batch, rvz_search_compact);
 * workgroups whose boards are all dead exit at once and leave their rows of logits / value / work
 * as they were. The row results do not
 * depend on the row's position in the batch (tests/test_gpu_network.py). stamps (nullable,
 * bench.py): every trunk workgroup w stores the device's 100 MHz wall clock (s_memrealtime) at its
 * start and end in stamps[2w], stamps[2w+1] (uint64 [rvz_resnet_h2_grid(board, filters, n)][2];
 * bits 56-63 of the end stamp: the workgroup's evaluated boards, 0 for a dead workgroup; bits
 * 52-55: the XCD it ran on):
 * max(end) - min(start) is the launch's span, readable after a replayed HIP graph (torch's HIP
 * runtime refuses external event records in stream capture). stamp_ctr (device uint32, nullable):
 * stamps is a ring of `ring` such launch rows and the trunk writes row *stamp_ctr % ring; the
 * heads launch given the same counter advances it by one (one thread, after the trunk is done),
 * so a replayed graph stamps every launch. */
int32_t rvz_resnet_h2_grid(int32_t board, int32_t filters, int32_t n);
int rvz_resnet_fwd_h2_ex(int32_t board, const float *x, int32_t n, const float *params,
                         const uint16_t *blob, int32_t filters, int32_t blocks, float *work,
                         float *logits, float *value, const int32_t *n_live, void *hip_stream);
int rvz_resnet_trunk_h2_ex(int32_t board, const float *x, int32_t n, const float *params,
                           const uint16_t *blob, int32_t filters, int32_t blocks, float *work,
                           const int32_t *n_live, uint64_t *stamps, const uint32_t *stamp_ctr,
                           int32_t ring, void *hip_stream);
int rvz_resnet_heads_fc_ex(int32_t board, const float *work, int32_t n, const float *params,
                           int32_t filters, int32_t blocks, float *logits, float *value,
                           const int32_t *n_live, uint32_t *stamp_ctr, void *hip_stream);

#ifdef __cplusplus
}
#endif
#endif /* RVZ_H */
