/*
 * rvz_oracle.h — CPU restatement of the reference's hot path (TEST INFRASTRUCTURE ONLY).
 *
 * This library is the parity oracle and the CPU baseline ("kind": "port") for the rvz engine.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and only as
 * the checker / the timed CPU baseline. The product path (alphazero-reversi_amd/) never links,
 * loads or calls anything here.
 *
 * It restates, literally and without the engine's optimisations (no leaf dedup, virtual loss kept,
 * Python/NumPy scalar typing reproduced), the behaviour of:
 *   /root/reference/src/game/board.py      Board        (rules, auto-pass, winner)
 *   /root/reference/src/game/game.py       ReversiGame  (make_move wrapper, canonical state)
 *   /root/reference/src/mcts/mcts.py       MCTSNode / MCTS.search / get_action_probs
 *   numpy 2.x legacy RandomState (MT19937 seed, random_sample, choice) and np.sum pairwise order.
 *
 * Parity of this oracle is pinned by the npz fixtures in tests/golden, generated from the importable Python
 * reference by tests/golden/make_golden.py.
 */
#ifndef RVZ_ORACLE_H
#define RVZ_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- board rules (board.py) ---- */
typedef struct {
    uint64_t black, white;
    int32_t side;    /* 1 = BLACK, 2 = WHITE: player to move (game.py:20, board.py:33) */
    int32_t over;    /* game_over */
    int32_t winner;  /* -1 = None, 0 = draw, 1 = BLACK, 2 = WHITE */
    int32_t passed;  /* passed_moves_in_a_row (board.py:37) */
} rvzo_game;

uint64_t rvzo_legal(int bs, uint64_t P, uint64_t O);
uint64_t rvzo_flips(int bs, int sq, uint64_t P, uint64_t O);
void rvzo_game_init(int bs, rvzo_game *g);
int rvzo_make_move(int bs, rvzo_game *g, int sq); /* sq = -1: pass; returns make_move's bool */
void rvzo_canonical(int bs, const rvzo_game *g, float *out /* [3, bs*bs] */);

/* ---- numpy legacy RNG + reductions ---- */
typedef struct { uint32_t key[624]; int32_t pos; } rvzo_mt;
void rvzo_mt_seed(rvzo_mt *s, uint32_t seed);
uint32_t rvzo_mt_next32(rvzo_mt *s);
double rvzo_mt_res53(rvzo_mt *s);
double rvzo_np_sum(const double *a, int n);
/* get_action_probs' tail (mcts.py:656-692): visits[npol] -> p[npol] (f64) and the chosen index.
 * *needs_draw tells whether np.random.choice would consume a random_sample; u is that sample. */
int rvzo_action(int npol, const int32_t *visits, double temperature, double u, double *p_out,
                int32_t *needs_draw);
int rvzo_action_needs_draw(int npol, const int32_t *visits, double temperature);

/* ---- batched reference-semantics search (mcts.py MCTS.search, one tree per game) ---- */
typedef struct rvzo_engine rvzo_engine;
rvzo_engine *rvzo_create(int bs, int n_games, int num_simulations, int batch_size, double c_puct);
void rvzo_destroy(rvzo_engine *e);
int rvzo_search_begin(rvzo_engine *e, const rvzo_game *roots);
/* Runs the traversals + pass 1 of the next batch for every game. Returns 1 when the search is
 * finished (nothing done), 0 otherwise. Per game: n_copies = queued leaf copies needing the NN,
 * leaf = their (shared) simulated game. Returns -1 if copies of one game disagree (dedup broken). */
int rvzo_search_step(rvzo_engine *e, rvzo_game *leaf, int32_t *n_copies);
int rvzo_search_submit(rvzo_engine *e, const float *probs /* [G, npol] */, const float *values);
int rvzo_search_visits(const rvzo_engine *e, int32_t *out /* [G, npol] */);
/* counters since create: traversals, summed traversal depth, expansions, terminal backups */
void rvzo_stats(const rvzo_engine *e, int64_t *out4);

#ifdef __cplusplus
}
#endif
#endif
