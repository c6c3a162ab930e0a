/*
 * rvz_oracle.c — CPU restatement of the reference hot path. TEST INFRASTRUCTURE ONLY
 * (parity checker + CPU baseline); see rvz_oracle.h for who may use it.
 *
 * Every function cites the reference lines it restates. Semantics are reproduced literally,
 * including the reference's quirks (no file masks in move generation, |d|-keyed flip masks,
 * stale UCB caches, BLACK-absolute terminal values, NumPy>=2 fp32 scalar promotion).
 */
#include "rvz_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------------ */
/* Board rules                                                                                 */
/* ------------------------------------------------------------------------------------------ */

static inline uint64_t sq_mask(int bs) {
    return bs * bs >= 64 ? ~0ULL : ((1ULL << (bs * bs)) - 1ULL);
}

static inline uint64_t shl_signed(uint64_t x, int s) {
    /* Python `(x << s)` for s > 0 else `x >> -s`; bits past 63 are dropped here, and in the
     * reference they are always ANDed with a 64-bit board right after, so this is identical. */
    return s > 0 ? (x << s) : (x >> (-s));
}

/* board.py:70-124 — get_valid_moves as a mask. NO file masks (the reference applies none), the
 * direction list is E,W,S,N,SE,NW,SW,NE as (dx,dy) with shift = dx + dy*size, 5 propagation steps. */
uint64_t rvzo_legal(int bs, uint64_t P, uint64_t O) {
    const int dirs[8][2] = {{1, 0}, {-1, 0}, {0, 1}, {0, -1}, {1, 1}, {-1, -1}, {-1, 1}, {1, -1}};
    uint64_t empty = ~(P | O) & sq_mask(bs); /* board.py:86 (64-bit mask; bs*bs bits here) */
    uint64_t valid = 0;
    for (int k = 0; k < 8; ++k) {
        int shift = dirs[k][0] + dirs[k][1] * bs;          /* board.py:104 */
        uint64_t cand = shl_signed(P, shift) & O;         /* board.py:108-111 */
        for (int i = 0; i < 5; ++i) cand |= shl_signed(cand, shift) & O; /* board.py:114-118 */
        valid |= shl_signed(cand, shift) & empty;         /* board.py:121-124 */
    }
    return valid;
}

/* board.py:189-219 — the flip walk. The edge mask is looked up by |d| (board.py:208), so W, NW
 * and SW use the east-side masks; this quirk is part of the reference semantics. */
uint64_t rvzo_flips(int bs, int sq, uint64_t P, uint64_t O) {
    const uint64_t not_col0 = bs == 8 ? 0xFEFEFEFEFEFEFEFEULL : 0;
    const uint64_t not_coln = bs == 8 ? 0x7F7F7F7F7F7F7F7FULL : 0;
    uint64_t m_nc0 = not_col0, m_ncn = not_coln;
    if (bs != 8) { /* build-defined generalisation for the 6x6 variant: same construction */
        m_nc0 = 0; m_ncn = 0;
        for (int r = 0; r < bs; ++r)
            for (int c = 0; c < bs; ++c) {
                if (c != 0) m_nc0 |= 1ULL << (r * bs + c);
                if (c != bs - 1) m_ncn |= 1ULL << (r * bs + c);
            }
    }
    const int dirs[8] = {1, -1, bs, -bs, bs - 1, -(bs - 1), bs + 1, -(bs + 1)}; /* board.py:193 */
    uint64_t move_bit = 1ULL << sq, flip = 0;
    for (int k = 0; k < 8; ++k) {
        int d = dirs[k], ad = d < 0 ? -d : d;
        uint64_t edge = ~0ULL;                                  /* .get(abs(d), all ones) */
        if (ad == 1 || ad == bs - 1) edge = m_nc0;              /* keys 1 and 7 */
        else if (ad == bs + 1) edge = m_ncn;                    /* key 9 */
        uint64_t line = 0, curr = move_bit;
        for (int step = 0; step < bs - 1; ++step) {             /* range(self.size - 1) */
            curr = shl_signed(curr, d);
            if (!(curr & O & edge)) break;
            line |= curr;
        }
        if (curr & P & edge) flip |= line;                      /* board.py:218-219 */
    }
    return flip;
}

void rvzo_game_init(int bs, rvzo_game *g) { /* board.py:25-39, game.py:11-26 */
    int m = bs / 2;
    g->white = (1ULL << ((m - 1) * bs + (m - 1))) | (1ULL << (m * bs + m));
    g->black = (1ULL << ((m - 1) * bs + m)) | (1ULL << (m * bs + (m - 1)));
    g->side = 1;
    g->over = 0;
    g->winner = -1;
    g->passed = 0;
}

static void determine_winner(rvzo_game *g) { /* board.py:363-373 */
    int b = __builtin_popcountll(g->black), w = __builtin_popcountll(g->white);
    g->winner = b > w ? 1 : (w > b ? 2 : 0);
}

/* game.py:36-70 wrapping board.py:135-251. sq = -1 is the pass move (-1, -1) (board.py:151-167);
 * any other sq outside [0, bs*bs) is an illegal move (returns 0, no state change). */
int rvzo_make_move(int bs, rvzo_game *g, int sq) {
    if (g->over) return 0;                                      /* game.py:47-48 */
    int player = g->side;
    uint64_t P = player == 1 ? g->black : g->white;
    uint64_t O = player == 1 ? g->white : g->black;
    if (sq == -1) {                                             /* board.py:151-167 */
        if (rvzo_legal(bs, P, O)) return 0;
        g->passed += 1;
        g->side = 3 - player;
        if (g->passed >= 2) {
            g->over = 1;
            determine_winner(g);
        }
        return 1;
    }
    if (sq < 0 || sq >= bs * bs) return 0;
    uint64_t mb = 1ULL << sq;
    if (!(mb & rvzo_legal(bs, P, O))) return 0;                 /* board.py:173-179 */
    uint64_t f = rvzo_flips(bs, sq, P, O);
    P ^= mb | f;                                                /* board.py:222-227 */
    O ^= f;
    if (player == 1) { g->black = P; g->white = O; } else { g->white = P; g->black = O; }
    g->side = 3 - player;                                       /* board.py:233 */
    g->passed = 0;                                              /* board.py:239 */
    uint64_t nP = g->side == 1 ? g->black : g->white, nO = g->side == 1 ? g->white : g->black;
    if (!rvzo_legal(bs, nP, nO)) {                              /* board.py:242-249 auto-pass */
        g->side = 3 - g->side;
        g->passed += 1;
        if (!rvzo_legal(bs, nO, nP)) {
            g->over = 1;
            determine_winner(g);
        }
    }
    return 1;
}

/* game.py:131-162: [current player's discs, opponent's discs, legal mask] as f32 planes. */
void rvzo_canonical(int bs, const rvzo_game *g, float *out) {
    int n = bs * bs;
    uint64_t P = g->side == 1 ? g->black : g->white, O = g->side == 1 ? g->white : g->black;
    uint64_t V = rvzo_legal(bs, P, O);
    for (int i = 0; i < n; ++i) {
        out[i] = (float)((P >> i) & 1);
        out[n + i] = (float)((O >> i) & 1);
        out[2 * n + i] = (float)((V >> i) & 1);
    }
}

/* ------------------------------------------------------------------------------------------ */
/* numpy legacy MT19937 (numpy/random/src/mt19937), random_sample, np.sum                      */
/* ------------------------------------------------------------------------------------------ */

void rvzo_mt_seed(rvzo_mt *s, uint32_t seed) { /* mt19937_seed == init_genrand */
    for (int pos = 0; pos < 624; ++pos) {
        s->key[pos] = seed;
        seed = 1812433253U * (seed ^ (seed >> 30)) + (uint32_t)(pos + 1);
    }
    s->pos = 624;
}

static void mt_gen(rvzo_mt *s) {
    const uint32_t UP = 0x80000000U, LO = 0x7fffffffU, A = 0x9908b0dfU;
    int i;
    uint32_t y;
    for (i = 0; i < 624 - 397; ++i) {
        y = (s->key[i] & UP) | (s->key[i + 1] & LO);
        s->key[i] = s->key[i + 397] ^ (y >> 1) ^ ((0U - (y & 1U)) & A);
    }
    for (; i < 623; ++i) {
        y = (s->key[i] & UP) | (s->key[i + 1] & LO);
        s->key[i] = s->key[i + 397 - 624] ^ (y >> 1) ^ ((0U - (y & 1U)) & A);
    }
    y = (s->key[623] & UP) | (s->key[0] & LO);
    s->key[623] = s->key[396] ^ (y >> 1) ^ ((0U - (y & 1U)) & A);
    s->pos = 0;
}

uint32_t rvzo_mt_next32(rvzo_mt *s) {
    if (s->pos == 624) mt_gen(s);
    uint32_t y = s->key[s->pos++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680U;
    y ^= (y << 15) & 0xefc60000U;
    y ^= (y >> 18);
    return y;
}

double rvzo_mt_res53(rvzo_mt *s) { /* legacy random_sample: genrand_res53 */
    uint32_t a = rvzo_mt_next32(s) >> 5, b = rvzo_mt_next32(s) >> 6;
    return ((double)a * 67108864.0 + (double)b) / 9007199254740992.0;
}

/* numpy pairwise_sum (loops_utils.h) for n <= 128: 8 accumulators, then the tail. */
double rvzo_np_sum(const double *a, int n) {
    if (n < 8) {
        double res = 0.0;
        for (int i = 0; i < n; ++i) res += a[i];
        return res;
    }
    if (n > 128) { /* recursive split at a multiple of 8 (not needed for npol <= 65) */
        int n2 = n / 2;
        n2 -= n2 % 8;
        return rvzo_np_sum(a, n2) + rvzo_np_sum(a + n2, n - n2);
    }
    double r[8];
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    int i;
    for (i = 8; i < n - (n % 8); i += 8)
        for (int j = 0; j < 8; ++j) r[j] += a[i + j];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i];
    return res;
}

/* numpy's `arr ** e` for a float64 array and a Python float exponent (fast_scalar_power). */
static double np_scalar_power(double x, double e) {
    if (e == 1.0) return x;
    if (e == 2.0) return x * x;
    if (e == 0.5) return sqrt(x);
    if (e == -1.0) return 1.0 / x;
    if (e == 0.0) return 1.0;
    return pow(x, e);
}

static int all_zero(const double *p, int n) {
    for (int i = 0; i < n; ++i)
        if (p[i] != 0.0) return 0;
    return 1;
}

/* mcts.py:656-692 after the search: visit counts -> probabilities -> temperature -> choice. */
static void action_probs(int npol, const int32_t *visits, double temperature, double *p) {
    int64_t total = 0;
    for (int i = 0; i < npol; ++i) total += visits[i];            /* mcts.py:663 */
    for (int i = 0; i < npol; ++i)
        p[i] = total > 0 ? (double)visits[i] / (double)total : 0.0; /* int/int true division */
    if (temperature > 0 && !all_zero(p, npol)) {                  /* mcts.py:673-676 */
        double t[128];
        double e = 1.0 / temperature;
        for (int i = 0; i < npol; ++i) t[i] = np_scalar_power(p[i], e);
        double s = rvzo_np_sum(t, npol);
        for (int i = 0; i < npol; ++i) p[i] = t[i] / s;
    }
}

int rvzo_action_needs_draw(int npol, const int32_t *visits, double temperature) {
    double p[128];
    action_probs(npol, visits, temperature, p);
    return !(temperature == 0.0 || all_zero(p, npol));
}

int rvzo_action(int npol, const int32_t *visits, double temperature, double u, double *p_out,
                int32_t *needs_draw) {
    action_probs(npol, visits, temperature, p_out);
    if (temperature == 0.0 || all_zero(p_out, npol)) {           /* mcts.py:679-681 argmax */
        int best = 0;
        for (int i = 1; i < npol; ++i)
            if (p_out[i] > p_out[best]) best = i;
        if (needs_draw) *needs_draw = 0;
        return best;
    }
    if (needs_draw) *needs_draw = 1;
    /* np.random.choice(npol, p=p): cdf = cumsum(p); cdf /= cdf[-1]; searchsorted(u, 'right') */
    double cdf[128];
    double acc = 0.0;
    for (int i = 0; i < npol; ++i) { acc += p_out[i]; cdf[i] = acc; }
    double last = cdf[npol - 1];
    int idx = 0;
    for (int i = 0; i < npol; ++i) {
        cdf[i] /= last;
        if (cdf[i] <= u) idx = i + 1;
    }
    return idx;
}

/* ------------------------------------------------------------------------------------------ */
/* Reference-semantics MCTS (mcts.py). One tree per game, literal traversals (no dedup).        */
/* ------------------------------------------------------------------------------------------ */

typedef struct {
    int32_t N, vl, first_child, nchild, turn, sq, has_valid, terminal, cache_valid, w_f32;
    double w;     /* value_sum: a Python float while w_f32 == 0, an np.float32 once w_f32 == 1 */
    double tv;    /* terminal_value (Python float) */
    float prior;  /* np.float32 from the softmax row */
    float cache;  /* cached_ucb (np.float32); initialised to -inf (mcts.py:69) */
    uint64_t valid;
} onode;

typedef struct {
    int32_t node;
    int32_t depth;      /* path = root .. node, length depth+1 */
    int32_t path[64];
    rvzo_game sim;
    int32_t needs_nn;
} oqueued;

typedef struct {
    onode *nodes;
    int32_t n_nodes, cap;
    rvzo_game root_game;
    int32_t active;
    oqueued *queue;     /* up to batch_size entries */
    int32_t n_queue;
} otree;

struct rvzo_engine {
    int bs, npol, G, S, B;
    double c_puct;
    int next_start;
    otree *t;
    int64_t stats[4];
};

rvzo_engine *rvzo_create(int bs, int n_games, int num_simulations, int batch_size, double c_puct) {
    if ((bs != 8 && bs != 6) || n_games <= 0 || num_simulations <= 0 || batch_size <= 0 ||
        batch_size > 4096)
        return NULL;
    rvzo_engine *e = (rvzo_engine *)calloc(1, sizeof(rvzo_engine));
    e->bs = bs;
    e->npol = bs * bs + 1;
    e->G = n_games;
    e->S = num_simulations;
    e->B = batch_size;
    e->c_puct = c_puct;
    e->next_start = num_simulations;
    e->t = (otree *)calloc((size_t)n_games, sizeof(otree));
    int n_batches = (num_simulations + batch_size - 1) / batch_size;
    for (int g = 0; g < n_games; ++g) {
        e->t[g].cap = 1 + n_batches * bs * bs;
        e->t[g].nodes = (onode *)malloc(sizeof(onode) * (size_t)e->t[g].cap);
        e->t[g].queue = (oqueued *)malloc(sizeof(oqueued) * (size_t)batch_size);
    }
    return e;
}

void rvzo_destroy(rvzo_engine *e) {
    if (!e) return;
    for (int g = 0; g < e->G; ++g) {
        free(e->t[g].nodes);
        free(e->t[g].queue);
    }
    free(e->t);
    free(e);
}

static void node_init(onode *n, float prior, int turn, int sq) { /* mcts.py:43-72 */
    memset(n, 0, sizeof(*n));
    n->prior = prior;
    n->turn = turn;
    n->sq = sq;
    n->first_child = -1;
    n->cache_valid = 1;            /* `cached_ucb = -inf` exists from __init__ on */
    n->cache = -INFINITY;
}

int rvzo_search_begin(rvzo_engine *e, const rvzo_game *roots) { /* mcts.py:332-341 */
    for (int g = 0; g < e->G; ++g) {
        otree *t = &e->t[g];
        t->root_game = roots[g];
        t->active = !roots[g].over;
        t->n_nodes = 1;
        t->n_queue = 0;
        onode *r = &t->nodes[0];
        node_init(r, 1.0f, roots[g].side, -1);
        uint64_t P = roots[g].side == 1 ? roots[g].black : roots[g].white;
        uint64_t O = roots[g].side == 1 ? roots[g].white : roots[g].black;
        r->has_valid = 1;          /* root gets game.get_valid_moves() at construction */
        r->valid = rvzo_legal(e->bs, P, O);
    }
    e->next_start = 0;
    return 0;
}

/* mcts.py:84-114 ucb_score, with NumPy>=2 scalar typing: prior is np.float32, so u and the sum
 * are float32; q is float32 once value_sum is (else a Python float, cast to f32 by the sum). */
static double ucb_score(onode *c, int parent_n, double c_puct) {
    if (c->N == 0) return INFINITY;
    if (c->cache_valid) return (double)c->cache;
    int visits = c->N + c->vl;
    float u = (float)c_puct * c->prior;
    u = u * (float)sqrt((double)parent_n);
    u = u / (float)(1 + visits);
    float s;
    int denom = c->N > 1 ? c->N : 1;
    if (c->w_f32) {
        float q = (float)c->w / (float)denom;
        if (c->turn != 1) q = -q;
        s = q + u;
    } else {
        double q = c->w / (double)denom;
        if (c->turn != 1) q = -q;
        s = (float)q + u;
    }
    c->cache = s;
    c->cache_valid = 1;
    return (double)s;
}

/* mcts.py:625-640 _backpropagate_path. value_is_f32 selects np.float32 (NN) vs Python float. */
static void backup(otree *t, const int32_t *path, int depth, double value, int value_is_f32) {
    int sign = 1;
    for (int k = depth; k >= 0; --k) {
        onode *n = &t->nodes[path[k]];
        if (n->vl > 0) n->vl -= 1;
        n->N += 1;
        if (value_is_f32) {
            float sv = (float)sign * (float)value;
            n->w = (double)((float)n->w + sv);
            n->w_f32 = 1;
        } else {
            double sv = sign * value;
            if (n->w_f32) n->w = (double)((float)n->w + (float)sv);
            else n->w = n->w + sv;
        }
        sign = -sign;
        n->cache_valid = 0;        /* `del node.cached_ucb` */
    }
}

/* mcts.py:409-444 _traverse on a copy of the root game. */
static int traverse(rvzo_engine *e, otree *t, oqueued *q) {
    int node = 0, depth = 0;
    q->sim = t->root_game;
    q->path[0] = 0;
    for (;;) {
        onode *n = &t->nodes[node];
        if (!((n->nchild > 0 || n->terminal) && !n->terminal)) break;
        n->vl += 1;
        int best_child = -1;
        double best = -INFINITY;
        for (int i = 0; i < n->nchild; ++i) {   /* children dict order = row-major insertion */
            int c = n->first_child + i;
            double s = ucb_score(&t->nodes[c], n->N, e->c_puct);
            if (s > best) { best = s; best_child = c; }
        }
        if (best_child < 0) return -1;           /* reference would call game.pass_turn(): dead */
        rvzo_make_move(e->bs, &q->sim, t->nodes[best_child].sq);
        node = best_child;
        q->path[++depth] = node;
        if (depth >= 63) return -1;
    }
    q->node = node;
    q->depth = depth;
    return 0;
}

int rvzo_search_step(rvzo_engine *e, rvzo_game *leaf, int32_t *n_copies) {
    if (e->next_start >= e->S) return 1;
    int bsz = e->S - e->next_start < e->B ? e->S - e->next_start : e->B; /* mcts.py:349 */
    int err = 0;
    int64_t st_trav = 0, st_depth = 0, st_term = 0;
#pragma omp parallel for schedule(dynamic, 16) reduction(| : err) reduction(+ : st_trav, st_depth, st_term)
    for (int g = 0; g < e->G; ++g) {
        otree *t = &e->t[g];
        n_copies[g] = 0;
        t->n_queue = 0;
        if (!t->active) continue;
        for (int k = 0; k < bsz; ++k) {                            /* mcts.py:355-386 */
            oqueued *q = &t->queue[t->n_queue];
            if (traverse(e, t, q)) { err |= 1; break; }
            st_trav += 1;
            st_depth += q->depth;
            onode *n = &t->nodes[q->node];
            if (n->terminal) {                                     /* mcts.py:364-366 */
                backup(t, q->path, q->depth, n->tv, 0);
                st_term += 1;
                continue;
            }
            t->n_queue++;
        }
        /* _process_batch pass 1 (mcts.py:561-585) */
        int first_nn = -1;
        for (int k = 0; k < t->n_queue; ++k) {
            oqueued *q = &t->queue[k];
            onode *n = &t->nodes[q->node];
            q->needs_nn = 0;
            if (!n->has_valid) {
                uint64_t P = q->sim.side == 1 ? q->sim.black : q->sim.white;
                uint64_t O = q->sim.side == 1 ? q->sim.white : q->sim.black;
                n->valid = rvzo_legal(e->bs, P, O);
                n->has_valid = 1;
            }
            if (!n->valid) {
                n->terminal = 1;
                int w = q->sim.over ? q->sim.winner : -1;          /* get_winner() */
                n->tv = w == 1 ? 1.0 : (w == 2 ? -1.0 : 0.0);
                backup(t, q->path, q->depth, n->tv, 0);
                st_term += 1;
                continue;
            }
            q->needs_nn = 1;
            if (first_nn < 0) {
                first_nn = k;
                leaf[g] = q->sim;
            } else if (q->node != t->queue[first_nn].node) {
                err |= 2; /* two distinct leaves in one batch: the engine's dedup would be wrong */
            }
            n_copies[g] += 1;
        }
    }
    e->stats[0] += st_trav;
    e->stats[1] += st_depth;
    e->stats[3] += st_term;
    e->next_start += e->B;
    return err ? -1 : 0;
}

/* _process_batch pass 2 (mcts.py:600-623): expand from the softmaxed row, then back up. */
int rvzo_search_submit(rvzo_engine *e, const float *probs, const float *values) {
    int64_t n_exp = 0;
#pragma omp parallel for schedule(dynamic, 16) reduction(+ : n_exp)
    for (int g = 0; g < e->G; ++g) {
        otree *t = &e->t[g];
        const float *row = probs + (size_t)g * e->npol;
        for (int k = 0; k < t->n_queue; ++k) {
            oqueued *q = &t->queue[k];
            if (!q->needs_nn) continue;
            onode *n = &t->nodes[q->node];
            if (n->terminal) continue;
            if (n->nchild == 0) {                                  /* MCTSNode.expand (:141-161) */
                int cnt = 0;
                n->first_child = t->n_nodes;
                for (int sq = 0; sq < e->bs * e->bs; ++sq) {
                    if (!((n->valid >> sq) & 1)) continue;
                    node_init(&t->nodes[t->n_nodes + cnt], row[sq], 3 - n->turn, sq);
                    cnt++;
                }
                n->nchild = cnt;
                t->n_nodes += cnt;
                n_exp += 1;
            }
            backup(t, q->path, q->depth, (double)values[g], 1);
        }
        t->n_queue = 0;
    }
    e->stats[2] += n_exp;
    return 0;
}

int rvzo_search_visits(const rvzo_engine *e, int32_t *out) { /* mcts.py:406-407 */
    for (int g = 0; g < e->G; ++g) {
        const otree *t = &e->t[g];
        int32_t *o = out + (size_t)g * e->npol;
        memset(o, 0, sizeof(int32_t) * (size_t)e->npol);
        const onode *r = &t->nodes[0];
        for (int i = 0; i < r->nchild; ++i) {
            const onode *c = &t->nodes[r->first_child + i];
            o[c->sq] = c->N;
        }
    }
    return 0;
}

void rvzo_stats(const rvzo_engine *e, int64_t *out4) {
    for (int i = 0; i < 4; ++i) out4[i] = e->stats[i];
}
