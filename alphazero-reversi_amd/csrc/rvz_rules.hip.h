// rvz_rules.hip.h — Reversi rules of the reference as gfx950 device functions.
//
// Semantics follow /root/reference/src/game/board.py exactly (bit-exact, including its quirks):
//  * move generation applies NO file masks (board.py:102-124), so lines wrap around the edges;
//  * the flip walk keys its edge mask by |d| (board.py:196-208), so W/NW/SW use east-side masks;
//  * a placement that flips nothing is legal if move generation says so;
//  * make_move auto-passes and ends the game inside the call (board.py:241-249).
// BS = 8 is the reference board; BS = 6 is the build-defined variant (same construction on a
// 6-stride bitboard).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rvz {

template <int BS>
struct Geo {
    static constexpr int NSQ = BS * BS;
    static constexpr int NPOL = NSQ + 1;
    static constexpr uint64_t FULL = NSQ == 64 ? ~0ull : ((1ull << NSQ) - 1ull);
    static constexpr uint64_t col_mask(int skip_col) {
        uint64_t m = 0;
        for (int r = 0; r < BS; ++r)
            for (int c = 0; c < BS; ++c)
                if (c != skip_col) m |= 1ull << (r * BS + c);
        return m;
    }
    static constexpr uint64_t NOT_COL0 = col_mask(0);        // 0xFEFE... for BS = 8
    static constexpr uint64_t NOT_COLN = col_mask(BS - 1);   // 0x7F7F... for BS = 8
    // black/white start squares (board.py:31-32 for BS = 8)
    static constexpr uint64_t START_WHITE =
        (1ull << ((BS / 2 - 1) * BS + (BS / 2 - 1))) | (1ull << ((BS / 2) * BS + BS / 2));
    static constexpr uint64_t START_BLACK =
        (1ull << ((BS / 2 - 1) * BS + BS / 2)) | (1ull << ((BS / 2) * BS + (BS / 2 - 1)));
};
static_assert(Geo<8>::NOT_COL0 == 0xFEFEFEFEFEFEFEFEull, "mask table");
static_assert(Geo<8>::NOT_COLN == 0x7F7F7F7F7F7F7F7Full, "mask table");
static_assert(Geo<8>::START_BLACK == 0x0000000810000000ull, "start position");
static_assert(Geo<8>::START_WHITE == 0x0000001008000000ull, "start position");

template <int S>
__device__ __forceinline__ uint64_t sh(uint64_t x) {
    if constexpr (S > 0) return x << S;
    else return x >> (-S);
}

// One direction of board.py:102-124: seed, 5 propagation steps, step onto an empty square.
template <int S>
__device__ __forceinline__ uint64_t legal_dir(uint64_t P, uint64_t O, uint64_t E) {
    uint64_t c = sh<S>(P) & O;
#pragma unroll
    for (int i = 0; i < 5; ++i) c |= sh<S>(c) & O;
    return sh<S>(c) & E;
}

template <int BS>
__device__ __forceinline__ uint64_t legal(uint64_t P, uint64_t O) {
    const uint64_t E = ~(P | O) & Geo<BS>::FULL;
    return legal_dir<1>(P, O, E) | legal_dir<-1>(P, O, E) | legal_dir<BS>(P, O, E) |
           legal_dir<-BS>(P, O, E) | legal_dir<BS + 1>(P, O, E) | legal_dir<-(BS + 1)>(P, O, E) |
           legal_dir<BS - 1>(P, O, E) | legal_dir<-(BS - 1)>(P, O, E);
}

// One direction of the flip walk (board.py:205-219) with the |d|-keyed edge mask.
template <int BS, int D>
__device__ __forceinline__ uint64_t flip_dir(uint64_t mb, uint64_t P, uint64_t O) {
    constexpr int AD = D < 0 ? -D : D;
    constexpr uint64_t EDGE = (AD == 1 || AD == BS - 1) ? Geo<BS>::NOT_COL0
                              : (AD == BS + 1 ? Geo<BS>::NOT_COLN : ~0ull);
    uint64_t line = 0, cur = mb;
#pragma unroll
    for (int s = 0; s < BS - 1; ++s) {
        cur = sh<D>(cur);
        if (!(cur & O & EDGE)) break;
        line |= cur;
    }
    return (cur & P & EDGE) ? line : 0ull;
}

template <int BS>
__device__ __forceinline__ uint64_t flips(int sq, uint64_t P, uint64_t O) {
    const uint64_t mb = 1ull << sq;
    return flip_dir<BS, 1>(mb, P, O) | flip_dir<BS, -1>(mb, P, O) | flip_dir<BS, BS>(mb, P, O) |
           flip_dir<BS, -BS>(mb, P, O) | flip_dir<BS, BS - 1>(mb, P, O) |
           flip_dir<BS, -(BS - 1)>(mb, P, O) | flip_dir<BS, BS + 1>(mb, P, O) |
           flip_dir<BS, -(BS + 1)>(mb, P, O);
}

// Game state of one ReversiGame (game.py keeps it in sync with its Board).
struct GameS {
    uint64_t black, white;
    int side;    // 1 BLACK, 2 WHITE
    int over;    // game_over
    int winner;  // -1 None, 0 draw, 1, 2
    int passed;  // passed_moves_in_a_row
};

__device__ __forceinline__ uint64_t mine(const GameS& g) { return g.side == 1 ? g.black : g.white; }
__device__ __forceinline__ uint64_t theirs(const GameS& g) { return g.side == 1 ? g.white : g.black; }

__device__ __forceinline__ void set_winner(GameS& g) {  // board.py:363-373
    const int b = __popcll(g.black), w = __popcll(g.white);
    g.winner = b > w ? 1 : (w > b ? 2 : 0);
}

// ReversiGame.make_move (game.py:36-70) -> Board.make_move (board.py:135-251).
// sq = -1: the pass move; any sq outside [0, NSQ) other than -1 is illegal (returns false).
template <int BS>
__device__ __forceinline__ bool make_move(GameS& g, int sq) {
    if (g.over) return false;
    const int player = g.side;
    uint64_t P = mine(g), O = theirs(g);
    if (sq == -1) {
        if (legal<BS>(P, O)) return false;
        g.passed += 1;
        g.side = 3 - player;
        if (g.passed >= 2) {
            g.over = 1;
            set_winner(g);
        }
        return true;
    }
    if (sq < 0 || sq >= Geo<BS>::NSQ) return false;
    const uint64_t mb = 1ull << sq;
    if (!(mb & legal<BS>(P, O))) return false;
    const uint64_t f = flips<BS>(sq, P, O);
    P ^= mb | f;
    O ^= f;
    if (player == 1) { g.black = P; g.white = O; } else { g.white = P; g.black = O; }
    g.side = 3 - player;
    g.passed = 0;
    if (!legal<BS>(O, P)) {          // new side to move (O) has no move: auto-pass
        g.side = player;
        g.passed += 1;
        if (!legal<BS>(P, O)) {
            g.over = 1;
            set_winner(g);
        }
    }
    return true;
}

// ---- wave-cooperative forms: lane l handles direction l & 7, an OR over each 8-lane group -------
// Every lane ends with the full result. Must be called with all 64 lanes active (DPP).
__device__ __forceinline__ uint32_t or8_u32(uint32_t x) {
    x |= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);   // quad_perm 1,0,3,2
    x |= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);   // quad_perm 2,3,0,1
    x |= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xF, 0xF, false);  // row_half_mirror
    return x;
}
__device__ __forceinline__ uint64_t or8_u64(uint64_t x) {
    return ((uint64_t)or8_u32((uint32_t)(x >> 32)) << 32) | or8_u32((uint32_t)x);
}

// direction d in [0, 8): E, W, S, N, SE, NW, SW, NE as a signed shift (board.py:89-98)
template <int BS>
__device__ __forceinline__ int dir_shift(int d) {
    const int a = d >> 1;
    const int mag = a == 0 ? 1 : (a == 1 ? BS : (a == 2 ? BS + 1 : BS - 1));
    return (d & 1) ? -mag : mag;
}

template <int BS>
__device__ __forceinline__ uint64_t legal_wave(uint64_t P, uint64_t O, int lane) {
    const int s = dir_shift<BS>(lane & 7);
    const int l = s > 0 ? s : 0, r = s > 0 ? 0 : -s;   // (x << l) >> r == sh(x, s)
    const uint64_t E = ~(P | O) & Geo<BS>::FULL;
    uint64_t c = ((P << l) >> r) & O;
#pragma unroll
    for (int i = 0; i < 5; ++i) c |= ((c << l) >> r) & O;
    return or8_u64(((c << l) >> r) & E);
}

template <int BS>
__device__ __forceinline__ uint64_t flips_wave(int sq, uint64_t P, uint64_t O, int lane) {
    const int s = dir_shift<BS>(lane & 7);
    const int l = s > 0 ? s : 0, r = s > 0 ? 0 : -s;
    const int ad = s > 0 ? s : -s;
    const uint64_t edge = (ad == 1 || ad == BS - 1) ? Geo<BS>::NOT_COL0
                          : (ad == BS + 1 ? Geo<BS>::NOT_COLN : ~0ull);
    uint64_t line = 0, cur = 1ull << sq;
    for (int k = 0; k < BS - 1; ++k) {
        cur = (cur << l) >> r;
        if (!(cur & O & edge)) break;
        line |= cur;
    }
    return or8_u64((cur & P & edge) ? line : 0ull);
}

// make_move with the wave-cooperative rules; same semantics as make_move<BS>.
template <int BS>
__device__ __forceinline__ bool make_move_wave(GameS& g, int sq, int lane) {
    if (g.over) return false;
    const int player = g.side;
    uint64_t P = mine(g), O = theirs(g);
    if (sq == -1) {
        if (legal_wave<BS>(P, O, lane)) return false;
        g.passed += 1;
        g.side = 3 - player;
        if (g.passed >= 2) {
            g.over = 1;
            set_winner(g);
        }
        return true;
    }
    if (sq < 0 || sq >= Geo<BS>::NSQ) return false;
    const uint64_t mb = 1ull << sq;
    if (!(mb & legal_wave<BS>(P, O, lane))) return false;
    const uint64_t f = flips_wave<BS>(sq, P, O, lane);
    P ^= mb | f;
    O ^= f;
    if (player == 1) { g.black = P; g.white = O; } else { g.white = P; g.black = O; }
    g.side = 3 - player;
    g.passed = 0;
    if (!legal_wave<BS>(O, P, lane)) {
        g.side = player;
        g.passed += 1;
        if (!legal_wave<BS>(P, O, lane)) {
            g.over = 1;
            set_winner(g);
        }
    }
    return true;
}

}  // namespace rvz
