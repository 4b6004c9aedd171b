// gc_core.h -- bitboard chess core for the batched env (gfx950 device code; also
// host-compilable so tests/ can differential-test it against the C oracle).
//
// Semantics are the reference engine's, /root/reference/src/lib.rs, NOT FIDE chess
// (SURVEY.md §0 Q1-Q10).  Square numbering is the reference's flat index
// sq = row*8 + col with row 0 = rank 8 (lib.rs:1235-1238); bit sq of a bitboard is
// that square.  Board state per lane: 7 bitboards (K,Q,R,B,N,P by type, both colours,
// plus white occupancy) and a 32-bit meta word.
//
// Every function is a pure function of its arguments (no tables, no memory):
// slider attacks use hyperbola quintessence with a full 64-bit bit reversal
// (v_bfrev_b32 x2), line masks are computed arithmetically, so one lane = one board
// needs no LDS and no cache traffic beyond its own state.
#pragma once
#include <type_traits>
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define GC_HD __host__ __device__ __forceinline__
#define GC_HDM __host__ __device__ __forceinline__
#else
#define GC_HD static inline
#define GC_HDM inline
#endif

namespace gc {

typedef uint64_t u64;
typedef uint32_t u32;

// ---- piece ids (lib.rs:11-17) and values (lib.rs:19-25) ------------------------
enum { EMPTY = 0, KING = 1, QUEEN = 2, ROOK = 3, BISHOP = 4, KNIGHT = 5, PAWN = 6 };
// actions (chess_v2.py:492-506)
enum { A_KSW = 4096, A_QSW = 4097, A_KSB = 4098, A_QSB = 4099, A_RESIGN = 4100, A_NONE = 0xFFFF };

// ---- meta word layout ----------------------------------------------------------
// bit 0      side to move (1 = WHITE)
// bits 1..4  castle rights wkc, wqc, bkc, bqc (as the reference's state dict stores them)
// bit 5      white_king_is_checked     bit 6  black_king_is_checked
// bit 7      env done flag (chess_v2.py self.done)
// bits 8..15 env move_count (chess_v2.py:194, 291-292; <= 150)
// bits 16..24 repetition-window length (<= 300)
enum : u32 {
    M_WHITE = 1u, M_WKC = 2u, M_WQC = 4u, M_BKC = 8u, M_BQC = 16u, M_RIGHTS = 30u,
    M_WCHK = 32u, M_BCHK = 64u, M_DONE = 128u,
    M_MC_SHIFT = 8, M_MC_MASK = 0xFFu << 8,
    M_HL_SHIFT = 16, M_HL_MASK = 0x1FFu << 16,
};

// ---- step reasons (per-ply info code) -------------------------------------------
enum { R_NONE = 0, R_MATE = 1, R_REPETITION = 2, R_MOVE_CAP = 3, R_NO_MOVES = 4, R_BOTH_CHECKED = 5,
       R_INVALID = 6, R_DONE_ALREADY = 7, R_MATED = 8, R_OPP_NO_MOVE = 9,
       R_WINDOW_FULL = 10 };

struct Pos {
    u64 k, q, r, b, n, p, w;  // by type (both colours) + white occupancy
    u32 meta;
};

static constexpr u64 FILE_A = 0x0101010101010101ull;  // col 0
static constexpr u64 FILE_H = 0x8080808080808080ull;  // col 7
static constexpr u64 DIAG = 0x8040201008040201ull;    // row == col
static constexpr u64 ANTI = 0x0102040810204080ull;    // row + col == 7

GC_HD int popc(u64 x) { return __builtin_popcountll(x); }
GC_HD int ctz(u64 x) { return __builtin_ctzll(x); }
GC_HD int msb(u64 x) { return 63 - __builtin_clzll(x); }
GC_HD u64 bit(int s) { return 1ull << s; }
// Three-input bitwise ops on bitboards: one v_bitop3_b32 per 32-bit half on gfx950 (truth
// table over a = 0xF0, b = 0xCC, c = 0xAA).  The compiler fuses few of these itself once the
// 64-bit ops are split into halves, and the Kogge-Stone fills and the set masks are chains of
// exactly this shape; the host build (CPU tests) evaluates the same expression in C.
template <unsigned TT>
GC_HD u64 bop3(u64 a, u64 b, u64 c) {
#if defined(__HIP_DEVICE_COMPILE__)
    const unsigned lo = __builtin_amdgcn_bitop3_b32((unsigned)a, (unsigned)b, (unsigned)c, TT);
    const unsigned hi = __builtin_amdgcn_bitop3_b32((unsigned)(a >> 32), (unsigned)(b >> 32), (unsigned)(c >> 32), TT);
    return ((u64)hi << 32) | lo;
#else
    u64 r = 0;
    for (int k = 0; k < 8; k++)
        if (TT >> k & 1) r |= ((k & 4) ? a : ~a) & ((k & 2) ? b : ~b) & ((k & 1) ? c : ~c);
    return r;
#endif
}
GC_HD u64 and_or(u64 a, u64 b, u64 c) { return bop3<0xEA>(a, b, c); }  // (a & b) | c
GC_HD u64 and3(u64 a, u64 b, u64 c) { return bop3<0x80>(a, b, c); }    // a & b & c
// squares below s (s < 64): shift-only, so no 64-bit subtract (a VCC carry chain, and on
// gfx950 a wait state before the carry is consumed)
GC_HD u64 below(int s) { return ~(~0ull << s); }

GC_HD u64 rbit(u64 x) {
#if defined(__clang__)
    return __builtin_bitreverse64(x);
#else
    x = ((x >> 1) & 0x5555555555555555ull) | ((x & 0x5555555555555555ull) << 1);
    x = ((x >> 2) & 0x3333333333333333ull) | ((x & 0x3333333333333333ull) << 2);
    x = ((x >> 4) & 0x0F0F0F0F0F0F0F0Full) | ((x & 0x0F0F0F0F0F0F0F0Full) << 4);
    return __builtin_bswap64(x);
#endif
}

GC_HD u64 occ_of(const Pos& s) { return s.k | s.q | s.r | s.b | s.n | s.p; }

// ---- line masks (arithmetic) ------------------------------------------------------
GC_HD u64 file_mask(int sq) { return FILE_A << (sq & 7); }
GC_HD u64 row_mask(int sq) { return 0xFFull << (sq & 56); }
GC_HD u64 diag_mask(int sq) {  // row - col = d
    int d = (sq >> 3) - (sq & 7);
    return d >= 0 ? DIAG << (8 * d) : DIAG >> (-8 * d);
}
GC_HD u64 anti_mask(int sq) {  // row + col = s
    int s = (sq >> 3) + (sq & 7);
    return s >= 7 ? ANTI << (8 * (s - 7)) : ANTI >> (8 * (7 - s));
}

// hyperbola quintessence on one line (mask includes the slider square).  The subtractions
// o - s and rbit(o) - rbit(s) are written as additions of -s = ~0 << sq and
// -rbit(s) = ~0 << (63 - sq): a 64-bit add is one instruction on gfx950 (v_lshl_add_u64),
// a 64-bit subtract is a carry pair through VCC plus a hazard wait state.
struct LineNeg {
    u64 s, neg, negr;
};
GC_HD LineNeg line_neg(int sq) { return LineNeg{bit(sq), ~0ull << sq, ~0ull << (63 - sq)}; }
GC_HD u64 line_att(u64 occ, u64 mask, const LineNeg& n) {
    u64 m = mask ^ n.s;
    u64 o = occ & m;
    u64 fwd = o + n.neg;
    u64 rev = rbit(o) + n.negr;
    return (fwd ^ rbit(rev)) & m;
}
GC_HD u64 rook_att(int sq, u64 occ) {
    LineNeg n = line_neg(sq);
    return line_att(occ, file_mask(sq), n) | line_att(occ, row_mask(sq), n);
}
GC_HD u64 bishop_att(int sq, u64 occ) {
    LineNeg n = line_neg(sq);
    return line_att(occ, diag_mask(sq), n) | line_att(occ, anti_mask(sq), n);
}
GC_HD u64 queen_att(int sq, u64 occ) {
    LineNeg n = line_neg(sq);
    return line_att(occ, file_mask(sq), n) | line_att(occ, row_mask(sq), n) | line_att(occ, diag_mask(sq), n) |
           line_att(occ, anti_mask(sq), n);
}

// leapers (set-wise; wrap masks per direction)
GC_HD u64 knight_set(u64 x) {
    u64 l1 = (x >> 1) & ~FILE_H, l2 = (x >> 2) & ~(FILE_H | (FILE_H >> 1));
    u64 r1 = (x << 1) & ~FILE_A, r2 = (x << 2) & ~(FILE_A | (FILE_A << 1));
    u64 h1 = l1 | r1, h2 = l2 | r2;
    return (h1 << 16) | (h1 >> 16) | (h2 << 8) | (h2 >> 8);
}
GC_HD u64 king_set(u64 x) {
    u64 h = ((x >> 1) & ~FILE_H) | ((x << 1) & ~FILE_A);
    u64 row = x | h;
    return h | (row << 8) | (row >> 8);
}
// pawn capture squares (r-p, c+1) and (r-p, c-1), p=+1 white (lib.rs:921-924)
GC_HD u64 pawn_att_set(u64 x, bool white) {
    return white ? (((x >> 7) & ~FILE_A) | ((x >> 9) & ~FILE_H))
                 : (((x << 9) & ~FILE_A) | ((x << 7) & ~FILE_H));
}

// in-between squares (exclusive) on a shared line, else 0 (branch-free, CPW formula)
GC_HD u64 between(int sq1, int sq2) {
    const u64 m1 = ~0ull;
    const u64 a2a7 = 0x0001010101010100ull;
    const u64 b2g7 = 0x0040201008040200ull;
    const u64 h1b7 = 0x0002040810204080ull;
    u64 btwn = (m1 << sq1) ^ (m1 << sq2);
    u64 file = (u64)((sq2 & 7) - (sq1 & 7));
    u64 rank = (u64)(((sq2 | 7) - sq1) >> 3);
    u64 line = ((file & 7) - 1) & a2a7;
    line += 2 * (((rank & 7) - 1) >> 58);
    line += (((rank - file) & 15) - 1) & b2g7;
    line += (((rank + file) & 15) - 1) & h1b7;
    line *= btwn & (0 - btwn);
    return line & btwn;
}
// the full line through a and b (a != b, aligned); isolates one pin segment from the union
GC_HD u64 line_through(int a, int b) {
    int dr = (b >> 3) - (a >> 3), dc = (b & 7) - (a & 7);
    if (dc == 0) return file_mask(a);
    if (dr == 0) return row_mask(a);
    if (dr == dc) return diag_mask(a);
    if (dr == -dc) return anti_mask(a);
    return 0;
}

// ---- piece lookup -------------------------------------------------------------------
GC_HD int type_at(const Pos& s, int sq) {
    u64 m = bit(sq);
    if (s.p & m) return PAWN;
    if (s.n & m) return KNIGHT;
    if (s.b & m) return BISHOP;
    if (s.r & m) return ROOK;
    if (s.q & m) return QUEEN;
    if (s.k & m) return KING;
    return EMPTY;
}
GC_HD int id_at(const Pos& s, int sq) {
    int t = type_at(s, sq);
    return (s.w >> sq) & 1 ? t : -t;
}
GC_HD void clear_sq(Pos& s, int sq) {
    u64 m = ~bit(sq);
    s.k &= m; s.q &= m; s.r &= m; s.b &= m; s.n &= m; s.p &= m; s.w &= m;
}
GC_HD void put(Pos& s, int sq, int id) {  // square must be clear
    if (id == 0) return;
    u64 m = bit(sq);
    int t = id < 0 ? -id : id;
    switch (t) {
        case KING: s.k |= m; break;
        case QUEEN: s.q |= m; break;
        case ROOK: s.r |= m; break;
        case BISHOP: s.b |= m; break;
        case KNIGHT: s.n |= m; break;
        default: s.p |= m; break;
    }
    if (id > 0) s.w |= m;
}

// ---- attack map of one side (lib.rs:669-677, attack mode, 1089-1104/1147-1174/928-933)
// Sliders stop at and include the first piece of either colour (so a slider ray ends AT a
// king: Q6); knights/kings every on-board target; pawns both diagonals except squares
// holding the pawn owner's own king (lib.rs:930).
// Kogge-Stone occluded fill of all sliders at once in one direction (shift by SH, left or
// right), then one more step: the attacked squares including the first blocker of either
// colour (attack-mode semantics).  `wrap` masks squares a step may not land on.
template <int SH, bool LEFT>
GC_HD u64 sh(u64 x) { return LEFT ? (x << SH) : (x >> SH); }
template <int SH, bool LEFT>
GC_HD u64 ray_fill_att(u64 gen, u64 empty, u64 wrap) {
    u64 pro = empty & wrap;
    gen = and_or(pro, sh<SH, LEFT>(gen), gen);
    pro &= sh<SH, LEFT>(pro);
    gen = and_or(pro, sh<2 * SH, LEFT>(gen), gen);
    pro &= sh<2 * SH, LEFT>(pro);
    gen = and_or(pro, sh<4 * SH, LEFT>(gen), gen);
    return sh<SH, LEFT>(gen) & wrap;
}
// the same fill's targets within a mask tm: sh(gen) & wrap & tm in one op per half
template <int SH, bool LEFT>
GC_HD u64 ray_fill_to(u64 gen, u64 empty, u64 wrap, u64 tm) {
    u64 pro = empty & wrap;
    gen = and_or(pro, sh<SH, LEFT>(gen), gen);
    pro &= sh<SH, LEFT>(pro);
    gen = and_or(pro, sh<2 * SH, LEFT>(gen), gen);
    pro &= sh<2 * SH, LEFT>(pro);
    gen = and_or(pro, sh<4 * SH, LEFT>(gen), gen);
    return and3(sh<SH, LEFT>(gen), wrap, tm);
}

// the map in three parts (the quad step kernel computes them on different waves)
GC_HD u64 side_attacks_leapers(const Pos& s, bool white) {
    u64 occ = occ_of(s);
    u64 mine = white ? s.w : (occ & ~s.w);
    return (pawn_att_set(s.p & mine, white) & ~(s.k & mine)) | knight_set(s.n & mine) | king_set(s.k & mine);
}
// branch-free for any number of sliders (a per-slider loop runs the wave's maximum)
GC_HD u64 side_attacks_orth(const Pos& s, bool white) {
    u64 occ = occ_of(s), empty = ~occ;
    u64 rq = (s.r | s.q) & (white ? s.w : (occ & ~s.w));
    return ray_fill_att<8, false>(rq, empty, ~0ull) | ray_fill_att<8, true>(rq, empty, ~0ull) |
           ray_fill_att<1, true>(rq, empty, ~FILE_A) | ray_fill_att<1, false>(rq, empty, ~FILE_H);
}
GC_HD u64 side_attacks_diag(const Pos& s, bool white) {
    u64 occ = occ_of(s), empty = ~occ;
    u64 bq = (s.b | s.q) & (white ? s.w : (occ & ~s.w));
    return ray_fill_att<7, false>(bq, empty, ~FILE_A) | ray_fill_att<9, false>(bq, empty, ~FILE_H) |
           ray_fill_att<9, true>(bq, empty, ~FILE_A) | ray_fill_att<7, true>(bq, empty, ~FILE_H);
}
GC_HD u64 side_attacks(const Pos& s, bool white) {
    return side_attacks_leapers(s, white) | side_attacks_orth(s, white) | side_attacks_diag(s, white);
}

// is square `sq` in `by_white`'s attack map? (the map membership test of lib.rs:661)
GC_HD bool sq_attacked(const Pos& s, int sq, bool by_white) {
    u64 occ = occ_of(s);
    u64 them = by_white ? s.w : (occ & ~s.w);
    u64 m = bit(sq);
    // pawn attack squares exclude squares holding the pawn owner's own king.  Branch-free:
    // lanes of a wave hold different boards, so early exits only add branch overhead.
    u64 pawns = (s.k & them & m) ? 0ull : (pawn_att_set(m, !by_white) & s.p & them);
    u64 att = pawns | (knight_set(m) & s.n & them) | (king_set(m) & s.k & them) |
              (rook_att(sq, occ) & (s.r | s.q) & them) | (bishop_att(sq, occ) & (s.b | s.q) & them);
    return att != 0;
}

// tracked king square of a colour, or -1 (lib.rs:641-653: the `break` leaves only the
// inner loop, so the LAST row holding a king wins, first column within it)
GC_HD int tracked_king(const Pos& s, bool white) {
    u64 occ = occ_of(s);
    u64 kk = s.k & (white ? s.w : (occ & ~s.w));
    u64 kz = kk ? kk : 1ull;  // branch-free: the result is discarded when there is no king
    int row = msb(kz) >> 3;
    int sq = ctz(kz & (0xFFull << (8 * row)));
    return kk ? sq : -1;
}

// The mover's check flag after a LEGAL `action` of the side `white` (update_state,
// lib.rs:1386-1393, for the side that just moved): s = the position before, ns = after.
//  * a non-king move: false.  The reference admits it only if king_is_checked(next_state)
//    is false (move_leaves_king_checked, lib.rs:612-624) -- the very flag computed here.
//  * a king move (the only own king): its target was outside the pre-move enemy map
//    (lib.rs:613-619), and vacating f / occupying t changes no leaper's attacks, so t is
//    attacked afterwards only (a) along the line through t and f by an enemy slider that had
//    the king on f in check (the Q6 retreat along the checking ray), or (b) by an enemy pawn,
//    when t held the enemy king: pawns skip squares holding their own king (lib.rs:930).
//  * castles and several own kings (tracked king may change): the full attack probe.
GC_HD bool mover_checked(const Pos& s, const Pos& ns, bool white, int action) {
    u64 occ0 = occ_of(s);
    u64 mine0 = white ? s.w : (occ0 & ~s.w);
    u64 kings = s.k & mine0;
    int f = (action >> 6) & 63, t = action & 63;
    bool kmove = action < 4096 && ((kings >> f) & 1);
    if (action >= 4096 || (kmove && (kings & (kings - 1)))) {  // rare: the general probe
        int mk = tracked_king(ns, white);
        return mk >= 0 && sq_attacked(ns, mk, !white);
    }
    if (!kmove) return false;
    u64 occn = occ_of(ns);
    u64 them = white ? (occn & ~ns.w) : ns.w;
    int dc = (t & 7) - (f & 7), dr = (t >> 3) - (f >> 3);
    bool orth = dc == 0 || dr == 0;
    u64 line = dc == 0 ? file_mask(f) : dr == 0 ? row_mask(f) : dr == dc ? diag_mask(f) : anti_mask(f);
    u64 sl = (orth ? (ns.r | ns.q) : (ns.b | ns.q)) & them;
    u64 att = line_att(occn, line, line_neg(f));
    u64 away = t > f ? below(f) : ~(below(f) | bit(f));  // beyond f, away from t
    u64 tb = bit(t);
    bool xray = (att & away & sl) != 0;
    bool pawn = (s.k & tb & ~mine0) && (pawn_att_set(tb, white) & ns.p & them);
    return xray || pawn;
}

// castle rights as the engine sees them on every call: State::new forces a colour's
// rights false when it has no king (lib.rs:315-322)
GC_HD u32 eff_rights(const Pos& s) {
    u64 occ = occ_of(s);
    u32 r = s.meta & M_RIGHTS;
    if (!(s.k & s.w)) r &= ~(M_WKC | M_WQC);
    if (!(s.k & occ & ~s.w)) r &= ~(M_BKC | M_BQC);
    return r;
}

// update_state (lib.rs:1386-1393): both check flags from the board
GC_HD u32 check_flags(const Pos& s) {
    u32 f = 0;
    int wk = tracked_king(s, true), bk = tracked_king(s, false);
    if (wk >= 0 && sq_attacked(s, wk, false)) f |= M_WCHK;
    if (bk >= 0 && sq_attacked(s, bk, true)) f |= M_BCHK;
    return f;
}

// ---- legal move generation context ----------------------------------------------------
struct Gen {
    u64 own, opp, occ;
    u64 checkmask;  // non-king targets must lie in it
    u64 pinned;     // own non-king pieces pinned to the tracked king
    u64 pinrays;    // union over pinners of between(king, pinner) | pinner
    u64 enemy_att;  // enemy attack map (king moves, castling); 0 if we have no king
    int ks;         // tracked king square or -1 (no legality filter)
    u32 castles;    // bit0 = queen side, bit1 = king side (reference order QS, KS)
    bool white;
    bool in_check;  // tracked king in the enemy attack map (_king_is_checked, lib.rs:634-667)
};

// Legality: the reference filters every non-king move by next_state + a full enemy
// attack-map recompute + "is my (tracked) king in it" (lib.rs:561, 612-632).  For
// en-passant-free rules that is exactly "target in checkmask AND (not pinned OR on the
// pin segment king..pinner)".  The segment, not the whole line: a pinned pawn's double
// push jumps blockers (Q1) and can land beyond its pinner or beyond its own king.  King
// moves are filtered by the pre-move enemy map instead (lib.rs:613-619, 1125-1128), which
// keeps the Q6 retreat-along-the-ray quirk.
// The context is built in three parts so that a pair of waves can share it (gymchess.hip,
// k_env_step2): gen_base (side, occupancy, tracked king), gen_pins (checkers, check mask,
// pins) and gen_enemy (enemy attack map, castles) -- the last two are independent.
GC_HD void gen_base(const Pos& s, Gen& g) {
    bool white = s.meta & M_WHITE;
    g.white = white;
    g.occ = occ_of(s);
    g.own = white ? s.w : (g.occ & ~s.w);
    g.opp = g.occ ^ g.own;
    g.ks = tracked_king(s, white);
    g.checkmask = ~0ull;
    g.pinned = 0;
    g.pinrays = 0;
    g.enemy_att = 0;
    g.castles = 0;
    g.in_check = false;
}

// Checkers, check mask and pins set-wise, one line through the king at a time (no loop over
// pinners, no `between`): a1 = the line's attack set from the king (up to and including the
// first blocker each way), a2 = the same with the own first blockers removed (the x-ray).
// Per direction (squares above / below the king): a slider of the line's kind at the end of
// a1 checks, and a1 on that side is "checker | between"; one at the end of a2 but not in a1
// pins the own blocker, and a2 on that side is the pin segment king..pinner (pinner included).
// Same sets as the reference's per-move filter (see above): a pinner is the first enemy piece
// on its ray with exactly one (own) piece between.
GC_HD void pin_line(u64 mask, const LineNeg& ln, u64 occ, u64 own, u64 sliders, u64 hi, u64 lo, u64& checkers,
                    u64& block, u64& pinned, u64& pinrays) {
    u64 a1 = line_att(occ, mask, ln);
    u64 a2 = line_att(occ ^ (a1 & own), mask, ln);
    u64 chk = a1 & sliders;
    u64 pn = a2 & ~a1 & sliders;
    checkers |= chk;
    u64 a1u = a1 & hi, a1d = a1 & lo, a2u = a2 & hi, a2d = a2 & lo;
    block |= ((a1u & chk) ? a1u : 0ull) | ((a1d & chk) ? a1d : 0ull);
    bool pu = (a2u & pn) != 0, pd = (a2d & pn) != 0;
    pinned |= ((pu ? a1u : 0ull) | (pd ? a1d : 0ull)) & own;
    pinrays |= (pu ? a2u : 0ull) | (pd ? a2d : 0ull);
}

// Partial pin / check sets of some of the four lines through the king (LINES bit 0 file,
// 1 rank, 2 diagonal, 3 anti-diagonal; LEAPERS: pawn / knight / king checkers), so that the
// quad step kernel can spread them over two waves; gen_pins_finish merges.
struct PinPart {
    u64 checkers, block, pinned, pinrays;
};
template <int LINES, bool LEAPERS>
GC_HD PinPart gen_pins_part(const Pos& s, const Gen& g) {
    PinPart p = {0, 0, 0, 0};
    if (g.ks < 0) return p;  // "King not present": no filter, no castling, no king moves
    int ks = g.ks;
    u64 kb = bit(ks);
    u64 opp = g.opp, occ = g.occ, own = g.own;
    if (LEAPERS)
        p.checkers = (pawn_att_set(kb, g.white) & s.p & opp) | (knight_set(kb) & s.n & opp) | (king_set(kb) & s.k & opp);
    u64 lo = below(ks), hi = ~(lo | kb);
    LineNeg ln = line_neg(ks);
    if (LINES & 3) {
        u64 rq = (s.r | s.q) & opp;
        if (LINES & 1) pin_line(file_mask(ks), ln, occ, own, rq, hi, lo, p.checkers, p.block, p.pinned, p.pinrays);
        if (LINES & 2) pin_line(row_mask(ks), ln, occ, own, rq, hi, lo, p.checkers, p.block, p.pinned, p.pinrays);
    }
    if (LINES & 12) {
        u64 bq = (s.b | s.q) & opp;
        if (LINES & 4) pin_line(diag_mask(ks), ln, occ, own, bq, hi, lo, p.checkers, p.block, p.pinned, p.pinrays);
        if (LINES & 8) pin_line(anti_mask(ks), ln, occ, own, bq, hi, lo, p.checkers, p.block, p.pinned, p.pinrays);
    }
    return p;
}
// The same sets from the enemy sliders ALIGNED with the king (a rook / queen on its file or
// rank, a bishop / queen on one of its diagonals), one at a time: with nothing between it and
// the king it checks (block += the squares between); with exactly one piece between, an own
// one, that piece is pinned and the segment king..slider is its pin ray.  (A second slider
// behind the first has two pieces between: neither checks nor pins -- the first-piece rule
// of the line form above.)  The loop runs the wave's largest aligned count, which under
// random play averages 0.17 per board and ~1.6 per 64-board wave (tools/pin_stats.py): an
// iteration of ~25 VALU ops against the ~440 of the four-line form.
// Everything the pins and the set-wise generation derive from the tracked king's square alone:
// its four lines and its leaper neighbourhoods (where an enemy pawn / knight / king checks it
// from).  A perft leaf counts ~35 children of one position whose side to move is the same in
// all of them and whose king did not move (the move was the other side's), so it computes this
// once per subtree root (perft2) instead of once per child.  ks < 0: no king (all zero but the
// masks of square 0, which nothing then uses: nothing is pinned).
// (The file and rank masks are two shifts each: recomputed where used, which keeps the perft
// leaf kernel's live registers down.)
struct KingLines {
    int ks;
    bool white;
    u64 kings;           // the side's kings the lines were computed for
    u64 dm, am;          // diagonal, anti-diagonal through the king
    u64 pawn, knight, king;  // squares from which an enemy pawn / knight / king attacks it
    GC_HDM u64 fm() const { return file_mask(ks < 0 ? 0 : ks); }
    GC_HDM u64 rm() const { return row_mask(ks < 0 ? 0 : ks); }
};
GC_HD KingLines king_lines(int ks, bool white, u64 kings = 0) {
    const int kq = ks < 0 ? 0 : ks;
    const u64 kb = ks < 0 ? 0ull : bit(ks);
    return KingLines{ks, white, kings, diag_mask(kq), anti_mask(kq), pawn_att_set(kb, white), knight_set(kb),
                     king_set(kb)};
}
// the lines of the side to move of s, with its kings recorded (the perft hint)
GC_HD KingLines king_lines_of(const Pos& s, bool white) {
    const u64 occ = occ_of(s), kings = s.k & (white ? s.w : (occ & ~s.w));
    return king_lines(tracked_king(s, white), white, kings);
}
// gen_base with the tracked king taken from a hint whose side and kings match (else searched)
GC_HD void gen_base_ks(const Pos& s, Gen& g, const KingLines& kh) {
    const bool white = s.meta & M_WHITE;
    g.white = white;
    g.occ = occ_of(s);
    g.own = white ? s.w : (g.occ & ~s.w);
    g.opp = g.occ ^ g.own;
    const u64 kings = s.k & g.own;
    g.ks = kh.ks;
    if (kings != kh.kings || white != kh.white) g.ks = tracked_king(s, white);
    g.checkmask = ~0ull;
    g.pinned = 0;
    g.pinrays = 0;
    g.enemy_att = 0;
    g.castles = 0;
    g.in_check = false;
}
GC_HD PinPart gen_pins_aligned_kl(const Pos& s, const Gen& g, const KingLines& kl) {
    PinPart p = {0, 0, 0, 0};
    if (g.ks < 0) return p;  // "King not present": no filter, no castling, no king moves
    const int ks = g.ks;
    const u64 opp = g.opp, occ = g.occ, own = g.own;
    p.checkers = (kl.pawn & s.p & opp) | (kl.knight & s.n & opp) | (kl.king & s.k & opp);
    const u64 fm = kl.fm(), rm = kl.rm(), dm = kl.dm, am = kl.am;
    u64 cand = ((s.r | s.q) & opp & (fm | rm)) | ((s.b | s.q) & opp & (dm | am));
    while (cand) {
        const int x = ctz(cand);
        cand &= cand - 1;
        const u64 xb = bit(x);
        const u64 line = (fm & xb) ? fm : (rm & xb) ? rm : (dm & xb) ? dm : am;
        const int lo = ks < x ? ks : x, hi = ks < x ? x : ks;
        const u64 btw = line & below(hi) & ~below(lo + 1);  // strictly between, on the line
        const u64 b = btw & occ;
        const bool clear = b == 0;
        const bool pin = b != 0 && (b & (b - 1)) == 0 && (b & own) != 0;
        p.checkers |= clear ? xb : 0ull;
        p.block |= clear ? btw : 0ull;
        p.pinned |= pin ? b : 0ull;
        p.pinrays |= pin ? (btw | xb) : 0ull;
    }
    return p;
}
GC_HD PinPart gen_pins_aligned(const Pos& s, const Gen& g) { return gen_pins_aligned_kl(s, g, king_lines(g.ks, g.white)); }
GC_HD void gen_pins_finish(Gen& g, const PinPart& p) {
    if (g.ks < 0) return;
    u64 checkers = p.checkers, block = p.block;
    g.in_check = checkers != 0;
    // one checker: capture it or block (checkers | between); two: king moves only; none: all
    g.checkmask = !checkers ? ~0ull : ((checkers & (checkers - 1)) ? 0ull : (checkers | block));
    g.pinned = p.pinned;
    g.pinrays = p.pinrays;
}
GC_HD void gen_pins(const Pos& s, Gen& g) { gen_pins_finish(g, gen_pins_aligned(s, g)); }

// castling (lib.rs:578-610 gate = OR of the colour's rights + king on board; geometry
// lib.rs:966-1056 tests the POSITIVE ids for black too: Q4), given g.enemy_att
GC_HD void gen_castles(const Pos& s, Gen& g) {
    if (g.ks < 0) return;
    bool white = g.white;
    u32 er = eff_rights(s);
    bool gate = white ? (er & (M_WKC | M_WQC)) : (er & (M_BKC | M_BQC));
    u64 wr = s.r & s.w, wk = s.k & s.w, A = g.enemy_att, occ = g.occ;
    int base = white ? 56 : 0;
    u64 qs_empty = 7ull << (base + 1), ks_empty = 3ull << (base + 5);
    u64 qs_safe = 7ull << (base + 2), ks_safe = 7ull << (base + 4);
    bool kpos = gate && (wk & bit(base + 4));
    bool qs = kpos && (wr & bit(base)) && !(occ & qs_empty) && !(A & qs_safe);
    bool kside = kpos && (wr & bit(base + 7)) && !(occ & ks_empty) && !(A & ks_safe);
    g.castles = (qs ? 1u : 0u) | (kside ? 2u : 0u);
}
GC_HD void gen_enemy(const Pos& s, Gen& g) {
    if (g.ks < 0) return;
    g.enemy_att = side_attacks(s, !g.white);
    gen_castles(s, g);
}

GC_HD void gen_init(const Pos& s, Gen& g) {
    gen_base(s, g);
    gen_pins(s, g);
    gen_enemy(s, g);
}

// pseudo targets (non-attack mode) of the own piece on `sq` of type `t`, before legality
GC_HD u64 pseudo_targets(const Pos& s, const Gen& g, int sq, int t) {
    u64 notown = ~g.own;
    switch (t) {
        case QUEEN: return queen_att(sq, g.occ) & notown;
        case ROOK: return rook_att(sq, g.occ) & notown;
        case BISHOP: return bishop_att(sq, g.occ) & notown;
        case KNIGHT: return knight_set(bit(sq)) & notown;
        case PAWN: {
            // lib.rs:935-958: one step if empty; two step from the start row if the
            // DESTINATION is empty (Q1); diagonal captures of any enemy piece (incl. king)
            u64 m = bit(sq), empty = ~g.occ, tg = 0;
            int row = sq >> 3;
            if (g.white) {
                tg |= (m >> 8) & empty;
                if (row == 6) tg |= (m >> 16) & empty;
            } else {
                tg |= (m << 8) & empty;
                if (row == 1) tg |= (m << 16) & empty;
            }
            return tg | (pawn_att_set(m, g.white) & g.opp);
        }
        default: return 0;
    }
}

// the squares on sq's side of the king ks (on any line through both): a pinned piece stays on
// its own pin segment.  pinrays is the union of every pinner's segment, and two pins can share
// a line (a rook behind the king, a queen in front); only a pawn's Q1 double push can cross its
// king -- onto the other pin's segment, where the move exposes the king (found by a 20 000-ply
// soak against the oracle, tools/soak.py)
GC_HD u64 king_side(int ks, int sq) { return sq > ks ? (ks >= 63 ? 0ull : ~below(ks + 1)) : below(ks); }

GC_HD u64 legal_targets(const Pos& s, const Gen& g, int sq, int t) {
    if (t == KING) return king_set(bit(sq)) & ~g.own & ~g.enemy_att;
    u64 tg = pseudo_targets(s, g, sq, t);
    if (g.ks < 0) return tg;
    tg &= g.checkmask;
    if (g.pinned & bit(sq)) tg &= g.pinrays & line_through(g.ks, sq) & king_side(g.ks, sq);
    return tg;
}

// attack-mode targets (get_possible_moves(attack=True), lib.rs:556-557)
GC_HD u64 attack_targets(const Pos& s, const Gen& g, int sq, int t) {
    u64 m = bit(sq);
    switch (t) {
        case KING: return king_set(m);
        case QUEEN: return rook_att(sq, g.occ) | bishop_att(sq, g.occ);
        case ROOK: return rook_att(sq, g.occ);
        case BISHOP: return bishop_att(sq, g.occ);
        case KNIGHT: return knight_set(m);
        case PAWN: return pawn_att_set(m, g.white) & ~(s.k & g.own);
        default: return 0;
    }
}

// ---- reference move ORDER within one piece ---------------------------------------------
// Returns the k-th target (0-based) of piece (sq, t) in the reference emission order.
//   K: (1,0),(-1,0),(0,1),(0,-1),(1,1),(1,-1),(-1,1),(-1,-1)   lib.rs:797-806
//   N: (-2,-1),(-2,1),(2,-1),(2,1),(-1,-2),(-1,2),(1,-2),(1,2)  lib.rs:891-900
//   P: one, two, (r-p,c+1), (r-p,c-1)                            lib.rs:921-958
//   R: rays (-1,0),(1,0),(0,-1),(0,1) outward                    lib.rs:835
//   B: rays (-1,-1),(-1,1),(1,-1),(1,1) outward                  lib.rs:845
//   Q: rook rays then bishop rays                                 lib.rs:824-831
GC_HD int kth_bit_desc(u64 x, int k) {
    for (int i = 0; i < k; i++) x &= ~bit(msb(x));
    return msb(x);
}
GC_HD int kth_bit_asc(u64 x, int k) {
    for (int i = 0; i < k; i++) x &= x - 1;
    return ctz(x);
}
GC_HD int ray_pick(u64 tg, int sq, u64 fm, u64 rm, u64 dm, u64 am, bool rook, bool bish, int& k) {
    // outward from sq: rays toward lower indices are walked high->low ("desc")
    u64 below = gc::below(sq), above = ~below & ~bit(sq);
#define GC_RAY(G, DESC)                                                      \
    {                                                                        \
        u64 gg = (G);                                                        \
        int c = popc(gg);                                                    \
        if (k < c) return DESC ? kth_bit_desc(gg, k) : kth_bit_asc(gg, k);  \
        k -= c;                                                              \
    }
    if (rook) {
        GC_RAY(tg & fm & below, true)   // (-1, 0)
        GC_RAY(tg & fm & above, false)  // (+1, 0)
        GC_RAY(tg & rm & below, true)   // (0, -1)
        GC_RAY(tg & rm & above, false)  // (0, +1)
    }
    if (bish) {
        GC_RAY(tg & dm & below, true)   // (-1, -1)
        GC_RAY(tg & am & below, true)   // (-1, +1)
        GC_RAY(tg & am & above, false)  // (+1, -1)
        GC_RAY(tg & dm & above, false)  // (+1, +1)
    }
#undef GC_RAY
    return -1;
}
// offsets packed as 8 signed bytes (no per-lane arrays -> no scratch memory)
GC_HD int offset_pick(u64 tg, int sq, u64 packed, int k) {
    for (int i = 0; i < 8; i++) {
        int t = sq + (int)(signed char)(packed >> (8 * i));
        if (t >= 0 && t < 64 && (tg >> t) & 1) {
            if (k == 0) return t;
            k--;
        }
    }
    return -1;
}
GC_HD u64 pack8(int a, int b, int c, int d, int e, int f, int g, int h) {
    return (u64)(uint8_t)a | (u64)(uint8_t)b << 8 | (u64)(uint8_t)c << 16 | (u64)(uint8_t)d << 24 |
           (u64)(uint8_t)e << 32 | (u64)(uint8_t)f << 40 | (u64)(uint8_t)g << 48 | (u64)(uint8_t)h << 56;
}
GC_HD int kth_target(u64 tg, int sq, int t, bool white, int k) {
    switch (t) {
        case KING: return offset_pick(tg, sq, pack8(8, -8, 1, -1, 9, 7, -7, -9), k);
        case KNIGHT: return offset_pick(tg, sq, pack8(-17, -15, 15, 17, -10, -6, 6, 10), k);
        case PAWN: return offset_pick(tg, sq, white ? pack8(-8, -16, -7, -9, 99, 99, 99, 99)
                                                    : pack8(8, 16, 9, 7, 99, 99, 99, 99), k);
        default: {
            bool rook = (t == ROOK || t == QUEEN), bish = (t == BISHOP || t == QUEEN);
            return ray_pick(tg, sq, file_mask(sq), row_mask(sq), diag_mask(sq), anti_mask(sq), rook, bish, k);
        }
    }
}

// f(target) for every target of the piece (type t) on sq in reference order -- kth_target's
// order in one pass: a leaper's offsets in order; a slider's rays in order, each outward
// (ascending bits above the square, descending below)
template <class F>
GC_HD void for_targets_ordered(u64 tg, int sq, int t, bool white, F&& f) {
    if (t == KING || t == KNIGHT || t == PAWN) {
        const u64 pk = t == KING ? pack8(8, -8, 1, -1, 9, 7, -7, -9)
                     : t == KNIGHT ? pack8(-17, -15, 15, 17, -10, -6, 6, 10)
                     : white ? pack8(-8, -16, -7, -9, 99, 99, 99, 99) : pack8(8, 16, 9, 7, 99, 99, 99, 99);
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const int to = sq + (int)(signed char)(pk >> (8 * j));
            if (to >= 0 && to < 64 && ((tg >> to) & 1)) f(to);
        }
    } else if (tg) {
        const u64 lo = below(sq), hi = ~lo & ~bit(sq);
        const bool rook = t == ROOK || t == QUEEN, bish = t == BISHOP || t == QUEEN;
        const u64 fm = file_mask(sq), rm = row_mask(sq), dm = diag_mask(sq), am = anti_mask(sq);
        const u64 ray[8] = {rook ? tg & fm & lo : 0, rook ? tg & fm & hi : 0, rook ? tg & rm & lo : 0,
                            rook ? tg & rm & hi : 0, bish ? tg & dm & lo : 0, bish ? tg & am & lo : 0,
                            bish ? tg & am & hi : 0, bish ? tg & dm & hi : 0};
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const bool desc = j == 0 || j == 2 || j == 4 || j == 5;  // toward lower indices: high -> low
            for (u64 m = ray[j]; m;) {
                const int to = desc ? msb(m) : ctz(m);
                f(to);
                m &= ~bit(to);
            }
        }
    }
}

// ---- whole-position enumeration --------------------------------------------------------
GC_HD int count_legal(const Pos& s, const Gen& g) {
    int n = 0;
    u64 pcs = g.own;
    while (pcs) {
        int sq = ctz(pcs);
        pcs ^= bit(sq);
        n += popc(legal_targets(s, g, sq, type_at(s, sq)));
    }
    return n + popc(g.castles);
}

// k-th legal action in reference order (normal moves row-major, castles QS then KS)
GC_HD int select_legal(const Pos& s, const Gen& g, int k) {
    u64 pcs = g.own;
    while (pcs) {
        int sq = ctz(pcs);
        pcs ^= bit(sq);
        int t = type_at(s, sq);
        u64 tg = legal_targets(s, g, sq, t);
        int c = popc(tg);
        if (k < c) return sq * 64 + kth_target(tg, sq, t, g.white, k);
        k -= c;
    }
    if (g.castles & 1) { if (k == 0) return g.white ? A_QSW : A_QSB; k--; }
    if (g.castles & 2) { if (k == 0) return g.white ? A_KSW : A_KSB; }
    return A_NONE;
}

// ---- type-uniform generation (the hot path) -------------------------------------------
// Lanes of a wave hold different boards, so a per-square loop that dispatches on the piece
// type serialises every type's code on every iteration.  Here each loop handles ONE piece
// type (lanes differ only in trip count) and pawns are done set-wise.  The targets of every
// other piece are parked in a per-lane scratch slot (LDS on the device) under the piece's
// ordinal among the side's pieces (its position in the row-major scan, lib.rs:510-511),
// and every piece's move count is recorded bit-sliced in 5 bitboards (cnt[b] bit sq = bit b
// of the count of the piece on sq), so a pick by rank needs no per-piece loop.
static constexpr int SCRATCH_SLOTS = 16;
static constexpr u64 ROW1 = 0xFFull << 8;   // black pawns' start row (lib.rs:947)
static constexpr u64 ROW6 = 0xFFull << 48;  // white pawns' start row (lib.rs:946)

struct MoveSet {
    u64 fastp;            // own pawns handled set-wise (the unpinned ones)
    u64 o1, o2, ol, orr;  // fast pawns with: single push, double push, capture c+1, capture c-1
    u64 cnt[5];           // bit-sliced per-square move counts (< 32) of all own pieces
    int total;            // legal move count including castles
    bool big;             // more own pieces than scratch slots: per-square fallback
};

struct NoScratch {  // count-only callers (perft leaves): no parking, no count planes
    static constexpr bool kPark = false;
    GC_HDM void put(int, u64) {}
    GC_HDM u64 get(int) const { return 0; }
};

GC_HD int ordinal(u64 own, int sq) { return popc(own & below(sq)); }

// a scratch type may keep its own per-piece counts (kPlanes = false: no bit-sliced planes)
template <class S, class = void>
struct planes_of {
    static constexpr bool value = S::kPark;
};
template <class S>
struct planes_of<S, decltype((void)S::kPlanes)> {
    static constexpr bool value = S::kPlanes;
};
template <class S>
GC_HD void park(MoveSet& ms, S& scr, u64 own, int sq, u64 tg, int& total) {
    int c = popc(tg);
    total += c;
    if (S::kPark) {
        scr.put(ordinal(own, sq), tg);
        if (planes_of<S>::value) {
#pragma unroll
            for (int b = 0; b < 5; b++) ms.cnt[b] |= (u64)((c >> b) & 1) << sq;  // no VCC select
        }
    }
}

GC_HD void moveset_clear(MoveSet& ms) {
    ms.fastp = ms.o1 = ms.o2 = ms.ol = ms.orr = 0;
#pragma unroll
    for (int b = 0; b < 5; b++) ms.cnt[b] = 0;
    ms.total = 0;
    ms.big = false;
}

// Rules = FIDE (gc_fide.h) reuses this generator with F = true: no king captures, the double
// step needs both squares empty, en passant for the pawns in ep_from (legality decided by
// fide::fgen).  Promotions are generated once per target (perft multiplies, gc_fide.h).
struct FideExtra {
    u64 ep_from;  // own pawns with a legal en-passant capture onto ep
    int ep;       // en-passant target square, or -1
};
GC_HD u64 fide_pawn_targets(const Pos& s, const Gen& g, int sq, const FideExtra& fx) {
    u64 m = bit(sq), empty = ~g.occ, notown = ~g.own & ~(s.k & g.opp);
    u64 one = g.white ? ((m >> 8) & empty) : ((m << 8) & empty);
    u64 two = g.white ? (((one & (0xFFull << 40)) >> 8) & empty) : (((one & (0xFFull << 16)) << 8) & empty);
    u64 tg = (one | two | (pawn_att_set(m, g.white) & g.opp)) & notown;
    if (g.ks >= 0) {
        tg &= g.checkmask;
        if (g.pinned & m) tg &= g.pinrays & line_through(g.ks, sq);
    }
    if (fx.ep_from & m) tg |= bit(fx.ep);
    return tg;
}

// Generator parts, one piece type each (the paired / quad step kernels run them on
// different waves).  Each ORs its pieces' counts into ms.cnt and returns its move count.
// Pawns, set-wise (lib.rs:935-958; Q1: the double push tests only the destination); the
// unpinned ones leave their four origin sets in ms (fastp, o1, o2, ol, orr).
template <class S, bool F = false>
GC_HD int gen_pawns(const Pos& s, const Gen& g, MoveSet& ms, S& scr, const FideExtra& fx = FideExtra{0, -1}) {
    const u64 own = g.own, cm = g.checkmask, nocap = F ? ~(s.k & g.opp) : ~0ull;  // FIDE: no king captures
    const u64 opp = g.opp & nocap;
    int total = 0;
    u64 P = s.p & own, fp = P & ~g.pinned, empty = ~g.occ;
    if (g.white) {
        ms.o1 = ((fp >> 8) & empty & cm) << 8;
        ms.o2 = F ? ((((((fp & ROW6) >> 8) & empty) >> 8) & empty & cm) << 16)
                  : ((((fp & ROW6) >> 16) & empty & cm) << 16);
        ms.ol = (((fp >> 7) & ~FILE_A) & opp & cm) << 7;
        ms.orr = (((fp >> 9) & ~FILE_H) & opp & cm) << 9;
    } else {
        ms.o1 = ((fp << 8) & empty & cm) >> 8;
        ms.o2 = F ? ((((((fp & ROW1) << 8) & empty) << 8) & empty & cm) >> 16)
                  : ((((fp & ROW1) << 16) & empty & cm) >> 16);
        ms.ol = (((fp << 9) & ~FILE_A) & opp & cm) >> 9;
        ms.orr = (((fp << 7) & ~FILE_H) & opp & cm) >> 7;
    }
    if (F && fx.ep >= 0) {  // en passant (legal by construction: fide::fgen)
        u64 epb = bit(fx.ep), ef = fx.ep_from & fp;
        ms.ol |= ef & (g.white ? ((epb & ~FILE_A) << 7) : ((epb & ~FILE_A) >> 9));
        ms.orr |= ef & (g.white ? ((epb & ~FILE_H) << 9) : ((epb & ~FILE_H) >> 7));
    }
    ms.fastp = fp;
    total += popc(ms.o1) + popc(ms.o2) + popc(ms.ol) + popc(ms.orr);
    if (planes_of<S>::value) {  // per-pawn counts o1+o2+ol+orr (0..4) as a bit-sliced sum
        u64 s1 = ms.o1 ^ ms.o2, c1 = ms.o1 & ms.o2, s2 = ms.ol ^ ms.orr, c2 = ms.ol & ms.orr;
        u64 b0 = s1 ^ s2, k0 = s1 & s2;
        ms.cnt[0] |= b0;
        ms.cnt[1] |= c1 ^ c2 ^ k0;
        ms.cnt[2] |= (c1 & c2) | (k0 & (c1 ^ c2));
    }
    u64 pp = P & g.pinned;  // pinned pawns: rare, per piece
    while (pp) {
        int sq = ctz(pp);
        pp ^= bit(sq);
        park(ms, scr, own, sq, F ? fide_pawn_targets(s, g, sq, fx) : legal_targets(s, g, sq, PAWN), total);
    }
    return total;
}
template <class S, bool F = false>
GC_HD int gen_knights(const Pos& s, const Gen& g, MoveSet& ms, S& scr) {
    const u64 own = g.own, notown_cm = ~own & g.checkmask & (F ? ~(s.k & g.opp) : ~0ull);
    int total = 0;
    u64 x = s.n & own;  // a pinned knight never has a move on its pin segment
    while (x) {
        int sq = ctz(x);
        x ^= bit(sq);
        park(ms, scr, own, sq, ((g.pinned >> sq) & 1) ? 0 : knight_set(bit(sq)) & notown_cm, total);
    }
    return total;
}
template <class S, bool F = false>
GC_HD int gen_kings(const Pos& s, const Gen& g, MoveSet& ms, S& scr) {
    const u64 own = g.own, nocap = F ? ~(s.k & g.opp) : ~0ull;
    int total = 0;
    u64 x = s.k & own;  // every own king; filtered by the pre-move enemy map only (lib.rs:613-619)
    while (x) {
        int sq = ctz(x);
        x ^= bit(sq);
        park(ms, scr, own, sq, king_set(bit(sq)) & ~own & ~g.enemy_att & nocap, total);
    }
    return total;
}
// sliders of one kind: T = QUEEN, ROOK or BISHOP
template <int T, class S, bool F = false>
GC_HD int gen_sliders(const Pos& s, const Gen& g, MoveSet& ms, S& scr) {
    const u64 own = g.own, notown_cm = ~own & g.checkmask & (F ? ~(s.k & g.opp) : ~0ull);
    int total = 0;
    u64 x = (T == QUEEN ? s.q : T == ROOK ? s.r : s.b) & own;
    while (x) {
        int sq = ctz(x);
        x ^= bit(sq);
        u64 tg = (T == QUEEN ? queen_att(sq, g.occ) : T == ROOK ? rook_att(sq, g.occ) : bishop_att(sq, g.occ)) & notown_cm;
        if ((g.pinned >> sq) & 1) tg &= g.pinrays & line_through(g.ks, sq);
        park(ms, scr, own, sq, tg, total);
    }
    return total;
}

// Part A of the generation: pawns (set-wise), knights, kings, queens.  `ms` cleared; ORs
// into ms.cnt; returns the number of moves found.  (The split A | B balances the two waves
// of the paired step kernel: queens cost a bishop plus a rook.)
template <class S, bool F = false>
GC_HD int gen_moves_a(const Pos& s, const Gen& g, MoveSet& ms, S& scr, const FideExtra& fx = FideExtra{0, -1}) {
    return gen_pawns<S, F>(s, g, ms, scr, fx) + gen_knights<S, F>(s, g, ms, scr) + gen_kings<S, F>(s, g, ms, scr) +
           gen_sliders<QUEEN, S, F>(s, g, ms, scr);
}

// Part B: bishops and rooks.  ORs into ms.cnt; returns the number of moves found.
template <class S, bool F = false>
GC_HD int gen_moves_b(const Pos& s, const Gen& g, MoveSet& ms, S& scr) {
    return gen_sliders<BISHOP, S, F>(s, g, ms, scr) + gen_sliders<ROOK, S, F>(s, g, ms, scr);
}

template <class S>
GC_HD void gen_moves(const Pos& s, const Gen& g, MoveSet& ms, S& scr) {
    moveset_clear(ms);
    ms.big = popc(g.own) > SCRATCH_SLOTS;
    if (ms.big) {
        ms.total = count_legal(s, g);
        return;
    }
    int total = popc(g.castles);
    total += gen_moves_a(s, g, ms, scr);
    total += gen_moves_b(s, g, ms, scr);
    ms.total = total;
}

// ---- set-wise generation in move-set order (the random self-play policy) ------------------
// Every legal move lies in exactly one of SW_SETS target bitboards, and the set fixes the way
// back from a target to its origin:
//   0-3   pawns: single push, double push (Q1), capture toward col+1, capture toward col-1
//   4-11  the eight knight jumps
//   12-15 rooks and queens, one bitboard per direction (row-1, row+1, col+1, col-1); 16-19
//         bishops and queens (row-1 col+1, row-1 col-1, row+1 col+1, row+1 col-1).  Within one
//         direction the rays of two sliders never overlap (the rear one's ray ends on the front
//         one), so a target has one origin: the first piece behind it in that direction
//   20-27 the eight king steps, filtered by the pre-move enemy map (lib.rs:613-619), for every
//         own king (boards with several kings: Q7)
// then the castles (queen side, king side).  A pinned piece joins only the sets of the
// directions along its pin line: a pinned slider's ray there ends at its king and at the
// pinner; a pinned pawn's targets are cut to its pin segment (a Q1 double push can jump the
// pinner); a pinned knight never moves.  The same legal moves as gen_moves (host test on fuzz
// positions); no per-piece loop, no parking, any number of pieces.  The policy's rank k is the
// k-th move in this order: sets by index, targets ascending within a set.
enum { SW_P1 = 0, SW_P2 = 1, SW_PL = 2, SW_PR = 3, SW_N = 4, SW_ORTH = 12, SW_DIAG = 16, SW_K = 20, SW_SETS = 28 };
struct MoveSets {
    u64 t[SW_SETS];
};
GC_HD int sw_popc(const u64* t, int lo, int hi) {
    int n = 0;
    for (int i = lo; i < hi; i++) n += popc(t[i]);
    return n;
}
// a square on the tracked king's lines (0 when there is no king: then nothing is pinned)
GC_HD int sw_ksq(const Gen& g) { return g.ks < 0 ? 0 : g.ks; }
GC_HD void sw_pawns_kl(const Pos& s, const Gen& g, const KingLines& kl, u64* t) {
    const u64 cm = g.checkmask, empty = ~g.occ, opp = g.opp, P = s.p & g.own, pr = g.pinrays;
    const u64 fp = P & ~g.pinned, pp = P & g.pinned;
    const u64 pf = pp & kl.fm(), pd = pp & kl.dm, pa = pp & kl.am;
    // a file-pinned pawn's double push stays on its side of the king (king_side): it crosses the
    // king exactly when the king stands on the square it jumps
    const u64 kb = bit(sw_ksq(g));
    if (g.white) {  // lib.rs:935-958, p = +1: toward row 0
        const u64 pf2 = ((pf & ~(kb << 8)) & ROW6) >> 16;
        t[SW_P1] = and3(and_or(pf >> 8, pr, fp >> 8), empty, cm);
        t[SW_P2] = and3(and_or(pf2, pr, (fp & ROW6) >> 16), empty, cm);
        t[SW_PL] = and3(and_or(pa >> 7, pr, fp >> 7), opp & ~FILE_A, cm);  // row-1 col+1: anti-diagonal
        t[SW_PR] = and3(and_or(pd >> 9, pr, fp >> 9), opp & ~FILE_H, cm);  // row-1 col-1: diagonal
    } else {
        const u64 pf2 = ((pf & ~(kb >> 8)) & ROW1) << 16;
        t[SW_P1] = and3(and_or(pf << 8, pr, fp << 8), empty, cm);
        t[SW_P2] = and3(and_or(pf2, pr, (fp & ROW1) << 16), empty, cm);
        t[SW_PL] = and3(and_or(pd << 9, pr, fp << 9), opp & ~FILE_A, cm);  // row+1 col+1: diagonal
        t[SW_PR] = and3(and_or(pa << 7, pr, fp << 7), opp & ~FILE_H, cm);  // row+1 col-1: anti-diagonal
    }
}
GC_HD void sw_pawns(const Pos& s, const Gen& g, u64* t) { sw_pawns_kl(s, g, king_lines(g.ks, g.white), t); }
// xm: extra target mask (FIDE: enemy kings are never captured)
GC_HD void sw_knights(const Pos& s, const Gen& g, u64* t, u64 xm = ~0ull) {
    const u64 N = s.n & g.own & ~g.pinned, tm = ~g.own & g.checkmask & xm;
    const u64 l1 = (N >> 1) & ~FILE_H, r1 = (N << 1) & ~FILE_A;
    const u64 l2 = (N >> 2) & ~(FILE_H | (FILE_H >> 1)), r2 = (N << 2) & ~(FILE_A | (FILE_A << 1));
    t[SW_N + 0] = (l1 << 16) & tm;  // target = origin + 15
    t[SW_N + 1] = (r1 << 16) & tm;  // + 17
    t[SW_N + 2] = (l1 >> 16) & tm;  // - 17
    t[SW_N + 3] = (r1 >> 16) & tm;  // - 15
    t[SW_N + 4] = (l2 << 8) & tm;   // + 6
    t[SW_N + 5] = (r2 << 8) & tm;   // + 10
    t[SW_N + 6] = (l2 >> 8) & tm;   // - 10
    t[SW_N + 7] = (r2 >> 8) & tm;   // - 6
}
GC_HD void sw_orth(const Pos& s, const Gen& g, u64* t, u64 xm = ~0ull) {
    const int kq = sw_ksq(g);
    const u64 S = (s.r | s.q) & g.own, fr = S & ~g.pinned, pp = S & g.pinned;
    const u64 empty = ~g.occ, tm = ~g.own & g.checkmask & xm;
    const u64 gf = fr | (pp & file_mask(kq)), gr = fr | (pp & row_mask(kq));
    t[SW_ORTH + 0] = ray_fill_to<8, false>(gf, empty, ~0ull, tm);
    t[SW_ORTH + 1] = ray_fill_to<8, true>(gf, empty, ~0ull, tm);
    t[SW_ORTH + 2] = ray_fill_to<1, true>(gr, empty, ~FILE_A, tm);
    t[SW_ORTH + 3] = ray_fill_to<1, false>(gr, empty, ~FILE_H, tm);
}
GC_HD void sw_diag(const Pos& s, const Gen& g, u64* t, u64 xm = ~0ull) {
    const int kq = sw_ksq(g);
    const u64 S = (s.b | s.q) & g.own, fr = S & ~g.pinned, pp = S & g.pinned;
    const u64 empty = ~g.occ, tm = ~g.own & g.checkmask & xm;
    const u64 gd = fr | (pp & diag_mask(kq)), ga = fr | (pp & anti_mask(kq));
    t[SW_DIAG + 0] = ray_fill_to<7, false>(ga, empty, ~FILE_A, tm);
    t[SW_DIAG + 1] = ray_fill_to<9, false>(gd, empty, ~FILE_H, tm);
    t[SW_DIAG + 2] = ray_fill_to<9, true>(gd, empty, ~FILE_A, tm);
    t[SW_DIAG + 3] = ray_fill_to<7, true>(ga, empty, ~FILE_H, tm);
}
// the diagonal sets SW_DIAG + lo .. SW_DIAG + hi - 1 only (the paired driver splits them
// between its two waves)
template <int lo, int hi>
GC_HD void sw_diag_part(const Pos& s, const Gen& g, u64* t, u64 xm = ~0ull) {
    const int kq = sw_ksq(g);
    const u64 S = (s.b | s.q) & g.own, fr = S & ~g.pinned, pp = S & g.pinned;
    const u64 empty = ~g.occ, tm = ~g.own & g.checkmask & xm;
    const u64 gd = fr | (pp & diag_mask(kq)), ga = fr | (pp & anti_mask(kq));
    if (lo <= 0 && 0 < hi) t[SW_DIAG + 0] = ray_fill_to<7, false>(ga, empty, ~FILE_A, tm);
    if (lo <= 1 && 1 < hi) t[SW_DIAG + 1] = ray_fill_to<9, false>(gd, empty, ~FILE_H, tm);
    if (lo <= 2 && 2 < hi) t[SW_DIAG + 2] = ray_fill_to<9, true>(gd, empty, ~FILE_A, tm);
    if (lo <= 3 && 3 < hi) t[SW_DIAG + 3] = ray_fill_to<7, true>(ga, empty, ~FILE_H, tm);
}
GC_HD void sw_kings(const Pos& s, const Gen& g, u64* t, u64 xm = ~0ull) {
    const u64 K = s.k & g.own, ok = ~g.own & ~g.enemy_att & xm;
    t[SW_K + 0] = (K >> 8) & ok;              // target = origin - 8
    t[SW_K + 1] = (K << 8) & ok;              // + 8
    t[SW_K + 2] = and3(K >> 1, ~FILE_H, ok);  // - 1
    t[SW_K + 3] = and3(K << 1, ~FILE_A, ok);  // + 1
    t[SW_K + 4] = and3(K >> 9, ~FILE_H, ok);  // - 9
    t[SW_K + 5] = and3(K >> 7, ~FILE_A, ok);  // - 7
    t[SW_K + 6] = and3(K << 7, ~FILE_H, ok);  // + 7
    t[SW_K + 7] = and3(K << 9, ~FILE_A, ok);  // + 9
}
// all sets of a position whose Gen is complete (gen_init); returns the move count
GC_HD int sw_gen(const Pos& s, const Gen& g, u64* t) {
    sw_pawns(s, g, t);
    sw_knights(s, g, t);
    sw_orth(s, g, t);
    sw_diag(s, g, t);
    sw_kings(s, g, t);
    return sw_popc(t, 0, SW_SETS) + popc(g.castles);
}
// ---- counting only (perft leaves, level expansion) ---------------------------------------
// gen_moves' total without parking anything, branch-free over the unpinned pieces: sliders
// of each kind set-wise, one Kogge-Stone fill per direction -- in one direction the rays of
// two own sliders never overlap (the rear one's ray ends on the front one), so the popcount
// of the union counts every (slider, target) pair once; knights per jump direction for the
// same reason (within one jump direction, knight -> target is one-to-one).  Pinned pieces
// (rare) and the kings one at a time, as gen_moves.  Any number of pieces (no slots).
template <int SH, bool LEFT>
GC_HD int ray_count(u64 gen, u64 empty, u64 wrap, u64 tmask) {
    return popc(ray_fill_to<SH, LEFT>(gen, empty, wrap, tmask));
}
// Pinned pieces need no loop either (the set-wise generation below, sw_*): a pinned slider
// fills only along its pin line -- its ray there ends at its king and at the pinner -- and a
// pinned pawn moves only along its pin line, cut to the pin segment (Q1); a pinned knight
// never moves.  So each direction's fill starts from the unpinned sliders plus the pinned ones
// on the king's line of that direction.
struct SliderGens {
    u64 f, r, d, a;  // generators of the file, rank, diagonal and anti-diagonal directions
};
GC_HD SliderGens slider_gens_kl(const Pos& s, const Gen& g, const KingLines& kl) {
    const u64 pin = g.pinned, oRQ = (s.r | s.q) & g.own, oBQ = (s.b | s.q) & g.own;
    const u64 fRQ = oRQ & ~pin, fBQ = oBQ & ~pin, pRQ = oRQ & pin, pBQ = oBQ & pin;
    return SliderGens{fRQ | (pRQ & kl.fm()), fRQ | (pRQ & kl.rm()), fBQ | (pBQ & kl.dm), fBQ | (pBQ & kl.am)};
}
GC_HD SliderGens slider_gens(const Pos& s, const Gen& g) { return slider_gens_kl(s, g, king_lines(g.ks, g.white)); }
// pawns (set-wise, pinned ones included), knights, kings (count_moves without the sliders)
GC_HD int count_nonsliders_kl(const Pos& s, const Gen& g, const KingLines& kl, bool kl_king = false,
                              const u64* ntab = nullptr) {
    const u64 own = g.own, tm = ~own & g.checkmask;
    int total = popc(g.castles);
    // pawns (lib.rs:935-958; Q1: the double push tests only the destination): sw_pawns' sets
    u64 pt[4];
    sw_pawns_kl(s, g, kl, pt);
    total += popc(pt[0]) + popc(pt[1]) + popc(pt[2]) + popc(pt[3]);
    // knights (a pinned knight never has a move on its pin segment)
    const u64 N = s.n & own & ~g.pinned;
    if (ntab) {  // (GC_PERFT_LDS=2: one table read per knight instead of the eight jump sets)
        for (u64 x = N; x; x &= x - 1) total += popc(ntab[ctz(x)] & tm);
    } else {
        const u64 l1 = (N >> 1) & ~FILE_H, r1 = (N << 1) & ~FILE_A;
        const u64 l2 = (N >> 2) & ~(FILE_H | (FILE_H >> 1)), r2 = (N << 2) & ~(FILE_A | (FILE_A << 1));
        total += popc((l1 << 16) & tm) + popc((r1 << 16) & tm) + popc((l1 >> 16) & tm) + popc((r1 >> 16) & tm) +
                 popc((l2 << 8) & tm) + popc((r2 << 8) & tm) + popc((l2 >> 8) & tm) + popc((r2 >> 8) & tm);
    }
    // kings: filtered by the pre-move enemy map only (lib.rs:613-619); several kings (Q7
    // boards, rare) one at a time
    const u64 K = s.k & own, ok = ~own & ~g.enemy_att;
    if (K & (K - 1)) {
        for (u64 x = K; x; x &= x - 1) total += popc(king_set(x & (0 - x)) & ok);
    } else {  // (kl_king: the lone king is the tracked one, its steps are kl.king)
        total += popc((kl_king && kl.ks >= 0 && K == bit(kl.ks) ? kl.king : king_set(K)) & ok);
    }
    return total;
}
GC_HD int count_nonsliders(const Pos& s, const Gen& g) { return count_nonsliders_kl(s, g, king_lines(g.ks, g.white)); }
GC_HD int count_moves(const Pos& s, const Gen& g) {
    const u64 tm = ~g.own & g.checkmask, empty = ~g.occ;
    const SliderGens G = slider_gens(s, g);
    return count_nonsliders(s, g) +
           ray_count<8, false>(G.f, empty, ~0ull, tm) + ray_count<8, true>(G.f, empty, ~0ull, tm) +
           ray_count<1, true>(G.r, empty, ~FILE_A, tm) + ray_count<1, false>(G.r, empty, ~FILE_H, tm) +
           ray_count<7, false>(G.a, empty, ~FILE_A, tm) + ray_count<9, false>(G.d, empty, ~FILE_H, tm) +
           ray_count<9, true>(G.d, empty, ~FILE_A, tm) + ray_count<7, true>(G.a, empty, ~FILE_H, tm);
}

// gen_init + count_moves of a position with the two Kogge-Stone passes fused: in each
// direction the enemy sliders' fill (the attack map) and the own unpinned sliders' fill (the
// count) share their propagator masks (the empty squares).  The perft leaves' child count.
template <int SH, bool LEFT>
GC_HD void ray_fill_pair(u64 ge, u64 go, u64 empty, u64 wrap, u64& ae, u64& ao) {
    u64 pro = empty & wrap;
    ge = and_or(pro, sh<SH, LEFT>(ge), ge);
    go = and_or(pro, sh<SH, LEFT>(go), go);
    pro &= sh<SH, LEFT>(pro);
    ge = and_or(pro, sh<2 * SH, LEFT>(ge), ge);
    go = and_or(pro, sh<2 * SH, LEFT>(go), go);
    pro &= sh<2 * SH, LEFT>(pro);
    ge = and_or(pro, sh<4 * SH, LEFT>(ge), ge);
    go = and_or(pro, sh<4 * SH, LEFT>(go), go);
    ae = sh<SH, LEFT>(ge) & wrap;
    ao = sh<SH, LEFT>(go) & wrap;
}
// kh: the king lines of the side to move if its tracked king sits on kh.ks (perft: computed
// once per subtree root); otherwise (a king captured, Q7) they are recomputed here
// ntab (the perft leaf's LDS table, round 5): the own knights' jumps by square instead of the
// eight shifted jump sets.  The own king's steps come from the per-root KingLines (perft 1.566 ->
// 1.583e12 same-box); the enemy king's neighbourhood from a table was measured slower.
GC_HD int count_position_kl(const Pos& s, const KingLines& kh, const u64* ntab = nullptr) {
    Gen g;
    gen_base_ks(s, g, kh);  // the tracked king from the hint while the side's kings are the hint's
    KingLines kl = kh;
    if (g.ks != kh.ks || g.white != kh.white) kl = king_lines(g.ks, g.white);
    gen_pins_finish(g, gen_pins_aligned_kl(s, g, kl));
    const u64 empty = ~g.occ, tm = ~g.own & g.checkmask;
    const u64 eRQ = (s.r | s.q) & g.opp, eBQ = (s.b | s.q) & g.opp;
    const SliderGens G = slider_gens_kl(s, g, kl);
    u64 att = 0, ae, ao;
    int n = 0;
#define GC_PAIR(SH, LEFT, GE, GO, WRAP)                  \
    ray_fill_pair<SH, LEFT>(GE, GO, empty, WRAP, ae, ao); \
    att |= ae;                                           \
    n += popc(ao & tm);
    GC_PAIR(8, false, eRQ, G.f, ~0ull)
    GC_PAIR(8, true, eRQ, G.f, ~0ull)
    GC_PAIR(1, true, eRQ, G.r, ~FILE_A)
    GC_PAIR(1, false, eRQ, G.r, ~FILE_H)
    GC_PAIR(7, false, eBQ, G.a, ~FILE_A)
    GC_PAIR(9, false, eBQ, G.d, ~FILE_H)
    GC_PAIR(9, true, eBQ, G.d, ~FILE_A)
    GC_PAIR(7, true, eBQ, G.a, ~FILE_H)
#undef GC_PAIR
    if (g.ks >= 0) {  // gen_enemy (no king: no map, no castling)
        g.enemy_att = att | side_attacks_leapers(s, !g.white);
        gen_castles(s, g);
    }
    return n + count_nonsliders_kl(s, g, kl, true, ntab);
}
GC_HD int count_position(const Pos& s) { return count_position_kl(s, king_lines_of(s, (s.meta & M_WHITE) != 0)); }

// ---- pick by rank in ACTION-ID order (the random self-play policy) ----------------------
// The driver draws k uniformly in [0, #legal); k maps to the k-th legal action in ascending
// action id (from*64+to, castles 4096.. last) -- the order of the legal-action mask, i.e.
// how a policy over the 4101-action space samples.  Any fixed bijection gives the same
// uniform policy; this one needs no per-piece loop: a 6-step binary search over the
// bit-sliced prefix counts finds the from-square, a 6-step popcount search the target.
GC_HD int prefix_count(const u64* cnt, u64 below) {
    return popc(cnt[0] & below) + 2 * popc(cnt[1] & below) + 4 * popc(cnt[2] & below) +
           8 * popc(cnt[3] & below) + 16 * popc(cnt[4] & below);
}
GC_HD int kth_set_bit(u64 x, int k) {  // 0-based, ascending; x has > k set bits
    int base = 0;
    u32 lo = (u32)x, c = (u32)__builtin_popcount(lo);
    u32 v = lo;
    if ((u32)k >= c) { k -= (int)c; v = (u32)(x >> 32); base = 32; }
#pragma unroll
    for (int w = 16; w; w >>= 1) {
        u32 m = (1u << w) - 1;
        int cc = __builtin_popcount(v & m);
        if (k >= cc) { k -= cc; v >>= w; base += w; }
    }
    return base;
}
GC_HD u64 fast_pawn_targets(const MoveSet& ms, int sq, bool white) {
    // origin-indexed move sets shifted onto the target squares, then isolated at sq's targets
    u64 m = bit(sq);
    u64 t1 = white ? ((ms.o1 & m) >> 8) : ((ms.o1 & m) << 8);
    u64 t2 = white ? ((ms.o2 & m) >> 16) : ((ms.o2 & m) << 16);
    u64 tl = white ? ((ms.ol & m) >> 7) : ((ms.ol & m) << 9);
    u64 tr = white ? ((ms.orr & m) >> 9) : ((ms.orr & m) << 7);
    return t1 | t2 | tl | tr;
}
template <class S>
GC_HD int select_action(const Pos& s, const Gen& g, const MoveSet& ms, const S& scr, int k) {
    int normal = ms.total - popc(g.castles);
    if (k >= normal) {  // castles: KS (4096 / 4098) sorts before QS (4097 / 4099)
        k -= normal;
        if (g.castles & 2) { if (k == 0) return g.white ? A_KSW : A_KSB; k--; }
        return g.white ? A_QSW : A_QSB;
    }
    if (ms.big) {  // per-square fallback (> SCRATCH_SLOTS own pieces)
        u64 pcs = g.own;
        while (pcs) {
            int sq = ctz(pcs);
            pcs ^= bit(sq);
            u64 tg = legal_targets(s, g, sq, type_at(s, sq));
            int c = popc(tg);
            if (k < c) return sq * 64 + kth_set_bit(tg, k);
            k -= c;
        }
        return A_NONE;
    }
    int lo = 0, pre = 0;  // largest square whose prefix count (squares below it) is <= k
#pragma unroll
    for (int step = 32; step; step >>= 1) {
        int p = prefix_count(ms.cnt, below(lo + step));
        bool take = p <= k;
        lo = take ? lo + step : lo;
        pre = take ? p : pre;  // the prefix at lo rides along: no seventh count
    }
    k -= pre;
    u64 parked = scr.get(ordinal(g.own, lo));  // both candidates, then a select (no branch)
    u64 tg = ((ms.fastp >> lo) & 1) ? fast_pawn_targets(ms, lo, g.white) : parked;
    return lo * 64 + kth_set_bit(tg, k);
}

// The same pick with short dependency chains (the rank search sits on the paired step's
// critical path): row totals of all 8 rows at once (per-byte popcounts of the 5 count planes,
// weighted), their byte-wise prefix sums by one multiply, a 3-step search over the 8 bytes;
// then the same over the 8 squares of the row (the planes' bits of that row spread to bytes).
// Byte sums need < 256 moves: more (never in play) take the bisection above.
GC_HD u64 byte_popc(u64 x) {
    x = x - ((x >> 1) & 0x5555555555555555ull);
    x = (x & 0x3333333333333333ull) + ((x >> 2) & 0x3333333333333333ull);
    return (x + (x >> 4)) & 0x0F0F0F0F0F0F0F0Full;
}
GC_HD u64 spread8(u32 b) {  // bit j of b -> byte j (0 / 1)
    u64 y = ((u64)(b & 0xFFu) * 0x0101010101010101ull) & 0x8040201008040201ull;
    return ((y + 0x7F7F7F7F7F7F7F7Full) >> 7) & 0x0101010101010101ull;
}
// p: inclusive prefix sums in 8 bytes (non-decreasing, byte 7 > k): the first byte above k
GC_HD int first_byte_above(u64 p, int k) {
    int r = (int)((p >> 24) & 0xFF) <= k ? 4 : 0;
    r += (int)((p >> (8 * r + 8)) & 0xFF) <= k ? 2 : 0;
    r += (int)((p >> (8 * r)) & 0xFF) <= k ? 1 : 0;
    return r;
}
template <class S>
GC_HD int select_action_swar(const Pos& s, const Gen& g, const MoveSet& ms, const S& scr, int k) {
    const int normal = ms.total - popc(g.castles);
    if (k >= normal || ms.big || normal > 255) return select_action(s, g, ms, scr, k);
    const u64 rows = byte_popc(ms.cnt[0]) + (byte_popc(ms.cnt[1]) << 1) + (byte_popc(ms.cnt[2]) << 2) +
                     (byte_popc(ms.cnt[3]) << 3) + (byte_popc(ms.cnt[4]) << 4);
    const u64 rpre = rows * 0x0101010101010101ull;
    const int r = first_byte_above(rpre, k);
    k -= r ? (int)((rpre >> (8 * r - 8)) & 0xFF) : 0;
    const int sh = 8 * r;
    const u64 sqs = spread8((u32)(ms.cnt[0] >> sh)) + (spread8((u32)(ms.cnt[1] >> sh)) << 1) +
                    (spread8((u32)(ms.cnt[2] >> sh)) << 2) + (spread8((u32)(ms.cnt[3] >> sh)) << 3) +
                    (spread8((u32)(ms.cnt[4] >> sh)) << 4);
    const u64 spre = sqs * 0x0101010101010101ull;
    const int f = first_byte_above(spre, k);
    k -= f ? (int)((spre >> (8 * f - 8)) & 0xFF) : 0;
    const int lo = sh + f;
    u64 parked = scr.get(ordinal(g.own, lo));
    u64 tg = ((ms.fastp >> lo) & 1) ? fast_pawn_targets(ms, lo, g.white) : parked;
    return lo * 64 + kth_set_bit(tg, k);
}

// origin of target `to` of set j.  Leapers: origin = to + a signed byte of four packed words
// (pawn offsets by colour); sliders: the nearest occupied square behind the target on the
// set's line (the squares between are empty: the ray came through them), branch-free.
GC_HD int sw_origin(const Gen& g, int j, int to) {
    const u64 w0 = g.white ? pack8(8, 16, 7, 9, -15, -17, 17, 15) : pack8(-8, -16, -9, -7, -15, -17, 17, 15);
    const u64 w1 = pack8(-6, -10, 10, 6, 0, 0, 0, 0), w2 = pack8(0, 0, 0, 0, 8, -8, 1, -1);
    const u64 w3 = pack8(9, 7, -7, -9, 0, 0, 0, 0);
    const int q = j >> 3;
    const u64 w = q == 0 ? w0 : q == 1 ? w1 : q == 2 ? w2 : w3;
    const int off = (int)(signed char)(w >> (8 * (j & 7)));
    // sliders: direction d = j - SW_ORTH; d 1, 2, 6, 7 move toward higher squares
    const int d = (j - SW_ORTH) & 7;
    const bool up = ((0xC6u >> d) & 1) != 0;
    const u64 line = d < 2 ? file_mask(to) : d < 4 ? row_mask(to) : (d == 5 || d == 6) ? diag_mask(to) : anti_mask(to);
    const u64 x = g.occ & line;
    const u64 lo = x & below(to), hi = x & (~below(to) ^ bit(to));
    const int sl = up ? (lo ? msb(lo) : 0) : (hi ? ctz(hi) : 0);
    const bool slider = j >= SW_ORTH && j < SW_K;
    return slider ? sl : to + off;
}
GC_HD int sw_select(const Gen& g, const u64* t, int k) {
    int j = SW_SETS;
    u64 tj = 0;
#pragma unroll
    for (int i = 0; i < SW_SETS; i++) {
        const int c = popc(t[i]);
        const bool hit = j == SW_SETS && k < c;
        j = hit ? i : j;
        tj = hit ? t[i] : tj;
        k = j == SW_SETS ? k - c : k;
    }
    if (j == SW_SETS) {  // castles: k is the rank among them
        if ((g.castles & 1) && k == 0) return g.white ? A_QSW : A_QSB;
        return g.white ? A_KSW : A_KSB;
    }
    const int to = kth_set_bit(tj, k);
    return sw_origin(g, j, to) * 64 + to;
}

// The same pick in two steps for the paired step kernel, whose sets sit in LDS: the sets'
// counts packed one byte per set into four words (set i in byte i % 8 of word i / 8), their
// prefix sums by three shift-adds per word, the set holding rank k by a word step and a byte
// step (no scan over 28 sets); then the caller fetches that one set and sw_finish turns the
// rank within it into the action.  Byte sums need < 256 moves (more: sw_select).
GC_HD void sw_pack(const u64* t, int lo, int hi, u64* cw) {
    for (int i = lo; i < hi; i++) cw[i >> 3] |= (u64)popc(t[i]) << (8 * (i & 7));
}
GC_HD u64 byte_prefix(u64 w) {  // inclusive prefix sums of the 8 bytes (no byte overflows)
    w += w << 8;
    w += w << 16;
    return w + (w << 32);
}
// rank k (< the sets' total) -> set index j and the rank within set j, with short dependency
// chains (it is the paired step's tail): the word from three independent compares against the
// running word totals; the byte as 8 - the number of byte prefixes > k, counted by a borrow-free
// compare of the bytes spread over 16-bit lanes.
GC_HD int sw_locate(const u64* cw, int& k) {
    const u64 p0 = byte_prefix(cw[0]), p1 = byte_prefix(cw[1]), p2 = byte_prefix(cw[2]), p3 = byte_prefix(cw[3]);
    const int c1 = (int)(p0 >> 56), c2 = c1 + (int)(p1 >> 56), c3 = c2 + (int)(p2 >> 56);
    const int w = (k >= c1) + (k >= c2) + (k >= c3);
    const u64 p = w == 0 ? p0 : w == 1 ? p1 : w == 2 ? p2 : p3;
    k -= w == 0 ? 0 : w == 1 ? c1 : w == 2 ? c2 : c3;
    const u64 H = 0x8000800080008000ull, K = (u64)(k + 1) * 0x0001000100010001ull, M = 0x00FF00FF00FF00FFull;
    const int above = popc((((p & M) | H) - K) & H) + popc(((((p >> 8) & M) | H) - K) & H);
    const int b = 8 - above;  // bytes with prefix <= k: the set is the next one
    k -= b ? (int)((p >> (8 * b - 8)) & 0xFF) : 0;
    return 8 * w + b;
}
GC_HD int sw_finish(const Gen& g, int j, u64 tj, int k) {
    const int to = kth_set_bit(tj, k);
    return sw_origin(g, j, to) * 64 + to;
}
GC_HD int sw_castle(const Gen& g, int k) {  // k: the rank among the castles
    if ((g.castles & 1) && k == 0) return g.white ? A_QSW : A_QSB;
    return g.white ? A_KSW : A_KSB;
}

// k-th legal action (0 <= k < ms.total) in reference order, from gen_moves' results
template <class S>
GC_HD int select_move(const Pos& s, const Gen& g, const MoveSet& ms, const S& scr, int k) {
    if (ms.big) return select_legal(s, g, k);
    u64 t[SCRATCH_SLOTS];
#pragma unroll
    for (int j = 0; j < SCRATCH_SLOTS; j++) t[j] = scr.get(j);  // all reads in flight at once
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
    for (int j = 0; j < SCRATCH_SLOTS; j++) asm volatile("" : "+v"(t[j]));  // one wait, not sixteen
#endif
    u64 pcs = g.own;
    int res = -1, rsq = 0, rk = 0;
    u64 rtg = 0;
    bool pawn = false;
#pragma unroll
    for (int j = 0; j < SCRATCH_SLOTS; j++) {  // predicated, fully unrolled scan in square order
        bool live = pcs != 0 && res < 0;
        int sq = pcs ? ctz(pcs) : 0;
        pcs &= pcs - 1;
        bool fast = (ms.fastp >> sq) & 1;
        int pc = (int)(((ms.o1 >> sq) & 1) + ((ms.o2 >> sq) & 1) + ((ms.ol >> sq) & 1) + ((ms.orr >> sq) & 1));
        int c = fast ? pc : popc(t[j]);
        bool hit = live && k < c;
        res = hit ? j : res;
        rsq = hit ? sq : rsq;
        rk = hit ? k : rk;
        rtg = hit ? t[j] : rtg;
        pawn = hit ? fast : pawn;
        k = (live && !hit) ? k - c : k;
    }
    if (res >= 0) {
        int sq = rsq;
        k = rk;
        if (pawn) {  // one, two, (r-p,c+1), (r-p,c-1)  (lib.rs:921-958)
            if ((ms.o1 >> sq) & 1) { if (k == 0) return sq * 64 + (g.white ? sq - 8 : sq + 8); k--; }
            if ((ms.o2 >> sq) & 1) { if (k == 0) return sq * 64 + (g.white ? sq - 16 : sq + 16); k--; }
            if ((ms.ol >> sq) & 1) { if (k == 0) return sq * 64 + (g.white ? sq - 7 : sq + 9); k--; }
            return sq * 64 + (g.white ? sq - 9 : sq + 7);
        }
        return sq * 64 + kth_target(rtg, sq, type_at(s, sq), g.white, k);
    }
    if (g.castles & 1) { if (k == 0) return g.white ? A_QSW : A_QSB; k--; }
    if (g.castles & 2) { if (k == 0) return g.white ? A_KSW : A_KSB; }
    return A_NONE;
}

// is `action` in the legal list? (chess_v2.py:240 `action not in self.possible_actions`)
GC_HD bool action_legal(const Pos& s, const Gen& g, int action) {
    if (action < 0 || action > A_RESIGN) return false;
    if (action >= 4096) {
        if (g.white) return (action == A_QSW && (g.castles & 1)) || (action == A_KSW && (g.castles & 2));
        return (action == A_QSB && (g.castles & 1)) || (action == A_KSB && (g.castles & 2));
    }
    int f = action >> 6, t = action & 63;
    if (!((g.own >> f) & 1)) return false;
    return (legal_targets(s, g, f, type_at(s, f)) >> t) & 1;
}

// action_legal(s, gen_init(s), action) without the whole enemy attack map: a non-king move
// needs the check mask and pins only, a king move the attack test of its one target (the
// map's bit there: sliders stop at the king still on its square, Q6), castles -- rare -- the
// full context.
GC_HD bool quick_legal(const Pos& s, int action) {
    if (action < 0 || action > A_RESIGN) return false;
    Gen g;
    gen_base(s, g);
    if (action >= 4096) {  // (castles read the enemy map, not the pins)
        gen_enemy(s, g);
        return action_legal(s, g, action);
    }
    const int f = action >> 6, t = action & 63;
    if (!((g.own >> f) & 1)) return false;
    const int ty = type_at(s, f);
    if (ty == KING) return ((king_set(bit(f)) & ~g.own) >> t & 1) && !sq_attacked(s, t, !g.white);
    gen_pins(s, g);
    return (legal_targets(s, g, f, ty) >> t) & 1;
}

// quick_legal in two independent halves (the quad API step validates on two waves at once):
// quick_legal(s, a) == quick_pseudo(s, a) && quick_safe(s, a) for every action a.
//  * quick_pseudo: the action id is in range, castles fully (action_legal), else the from-square
//    holds an own piece and the target is among its pseudo targets -- every piece type tested
//    branch-free (lanes hold different types: a switch would run every case), sliders by the
//    line and the squares strictly between; a king's step without the attack test;
//  * quick_safe: a king step's target not attacked (sq_attacked: the map with the king still on
//    its square, Q6); any other move inside the check mask and on its pin segment; castles and
//    out-of-range ids true (quick_pseudo decides them).
GC_HD bool quick_pseudo(const Pos& s, int action) {
    if (action < 0 || action > A_RESIGN) return false;
    Gen g;
    gen_base(s, g);
    if (action >= 4096) {  // (castles read the enemy map, not the pins)
        gen_enemy(s, g);
        return action_legal(s, g, action);
    }
    const int f = action >> 6, t = action & 63;
    const u64 fb = bit(f), tb = bit(t);
    const int ty = type_at(s, f);
    const int df = (t & 7) - (f & 7), dr = (t >> 3) - (f >> 3);
    const bool orth = (df == 0) != (dr == 0);
    const bool dia = df != 0 && (df == dr || df == -dr);
    const bool clear = (between(f, t) & g.occ) == 0;
    const u64 empty = ~g.occ;
    // pawns (lib.rs:935-958): one step, two from the start row (Q1: the destination only), a
    // diagonal capture of any enemy piece
    const u64 push = g.white ? (((fb >> 8) | ((fb & ROW6) >> 16)) & empty) : (((fb << 8) | ((fb & ROW1) << 16)) & empty);
    const u64 pawn = push | (pawn_att_set(fb, g.white) & g.opp);
    const u64 leap = (ty == KNIGHT ? knight_set(fb) : king_set(fb)) & ~g.own;
    const bool ok = ty == PAWN ? (pawn & tb) != 0
                  : (ty == KNIGHT || ty == KING) ? (leap & tb) != 0
                  : ty == QUEEN ? (orth || dia) && clear
                  : ty == ROOK ? orth && clear
                  : ty == BISHOP ? dia && clear : false;
    return ((g.own >> f) & 1) && ok && (ty == PAWN || !(g.own & tb));
}
GC_HD bool quick_safe(const Pos& s, int action) {
    if (action < 0 || action >= 4096) return true;
    const int f = action >> 6, t = action & 63;
    Gen g;
    gen_base(s, g);
    if (type_at(s, f) == KING) return !sq_attacked(s, t, !g.white);
    gen_pins(s, g);
    if (g.ks < 0) return true;
    u64 tg = g.checkmask;
    if (g.pinned & bit(f)) tg &= g.pinrays & line_through(g.ks, f) & king_side(g.ks, f);
    return (tg >> t) & 1;
}

// ---- transition: next_state (lib.rs:679-784) ------------------------------------------
// `white_player` is the caller's player argument (it selects promotion colour and which
// rights are revoked), not necessarily the piece's colour.  Returns 0 ok, -1 if the from
// square is empty (the reference panics), -2 bad action.  *reward = captured value
// (+10 on the dead promotion branch); *irrev = pawn move or capture (repetition window).
GC_HD int apply_move(Pos& s, bool white_player, int action, int* reward, bool* irrev) {
    // piece values by |id| (lib.rs:19-25) as 4-bit fields: 0,0,10,5,3,3,1 -- no memory table
    *reward = 0;
    *irrev = false;
    if (action < 4096) {
        int f = action >> 6, t = action & 63;
        int pid = id_at(s, f);
        if (pid == 0) return -1;
        int cid = id_at(s, t);
        int pt = pid < 0 ? -pid : pid, ct = cid < 0 ? -cid : cid;
        clear_sq(s, f);
        clear_sq(s, t);
        int nid = pid;
        *reward = (int)((0x1335A00u >> (4 * ct)) & 0xFu);
        if (pt == PAWN && ((white_player && (t >> 3) == 7) || (!white_player && (t >> 3) == 0))) {
            nid = white_player ? QUEEN : -QUEEN;  // QUEEN_ID * player (lib.rs:706)
            *reward += 10;
        }
        put(s, t, nid);
        *irrev = (pt == PAWN) || (cid != 0);
        if (pid == KING) {  // positive id only (Q5)
            s.meta &= white_player ? ~(u32)(M_WKC | M_WQC) : ~(u32)(M_BKC | M_BQC);
        } else if (pid == ROOK) {
            if ((f & 7) == 0) s.meta &= white_player ? ~(u32)M_WQC : ~(u32)M_BQC;
            else if ((f & 7) == 7) s.meta &= white_player ? ~(u32)M_WKC : ~(u32)M_BKC;
        }
    } else {
        switch (action) {  // lib.rs:740-773
            case A_KSW:
                clear_sq(s, 60); clear_sq(s, 61); clear_sq(s, 62); clear_sq(s, 63);
                put(s, 61, ROOK); put(s, 62, KING);
                s.meta &= ~(u32)(M_WKC | M_WQC);
                break;
            case A_QSW:
                clear_sq(s, 56); clear_sq(s, 57); clear_sq(s, 58); clear_sq(s, 59); clear_sq(s, 60);
                put(s, 58, KING); put(s, 59, ROOK);
                s.meta &= ~(u32)(M_WKC | M_WQC);
                break;
            case A_KSB:
                clear_sq(s, 4); clear_sq(s, 5); clear_sq(s, 6); clear_sq(s, 7);
                put(s, 5, -ROOK); put(s, 6, -KING);
                s.meta &= ~(u32)(M_BKC | M_BQC);
                break;
            case A_QSB:
                clear_sq(s, 0); clear_sq(s, 1); clear_sq(s, 2); clear_sq(s, 3); clear_sq(s, 4);
                put(s, 2, -KING); put(s, 3, -ROOK);
                s.meta &= ~(u32)(M_BKC | M_BQC);
                break;
            default: return -2;
        }
    }
    // current_player = other (lib.rs:778-780)
    s.meta = white_player ? (s.meta & ~(u32)M_WHITE) : (s.meta | M_WHITE);
    return 0;
}

// next_state for a LEGAL move of the side to move (the env's case: the player owns the
// piece), branch-free.  Same result as apply_move for such moves: the promotion branch is
// unreachable (a pawn of the mover never reaches the row lib.rs:703-704 tests), a white king
// move revokes both white rights, a white rook leaving column 0 / 7 revokes one (Q5).
GC_HD void apply_legal(Pos& s, bool white, int action, int* reward, bool* irrev) {
    // castles (lib.rs:740-773) in the same branch-free form: the king's and rook's squares
    // (and the ones between) cleared, king and rook put on their targets in the colour of the
    // castle id; both rights of that colour revoked
    const bool cs = action >= 4096;
    const bool cw = action == A_KSW || action == A_QSW, cks = action == A_KSW || action == A_KSB;
    const int base = cw ? 56 : 0;
    const u64 cclr = cks ? (0xFull << (base + 4)) : (0x1Full << base);
    const u64 ck = cs ? bit(base + (cks ? 6 : 2)) : 0ull, cr = cs ? bit(base + (cks ? 5 : 3)) : 0ull;
    int f = (action >> 6) & 63, t = action & 63;
    u64 fm = cs ? 0ull : bit(f), tm = cs ? 0ull : bit(t), clr = cs ? ~cclr : ~(fm | tm);
    // captured value (lib.rs:19-25, 698): Q 10, R 5, B/N 3, P 1, K 0
    // the target holds at most one piece: a sum of bit tests, no branch chain
    int v = 10 * (int)((s.q >> t) & 1) + 5 * (int)((s.r >> t) & 1) + 3 * (int)(((s.b | s.n) >> t) & 1) +
            (int)((s.p >> t) & 1);
    *reward = cs ? 0 : v;
    *irrev = !cs && (((s.p & fm) != 0) || ((occ_of(s) & tm) != 0));
    bool wk = (s.k & s.w & fm) != 0, wr = (s.r & s.w & fm) != 0;
#define GC_MV(X) s.X = (s.X & clr) | ((s.X & fm) ? tm : 0ull)
    GC_MV(k); GC_MV(q); GC_MV(r); GC_MV(b); GC_MV(n); GC_MV(p); GC_MV(w);
#undef GC_MV
    s.k |= ck;
    s.r |= cr;
    s.w |= cw ? (ck | cr) : 0ull;
    u32 clear = (wk ? (u32)(M_WKC | M_WQC) : 0u) | ((wr && (f & 7) == 0) ? (u32)M_WQC : 0u) |
                ((wr && (f & 7) == 7) ? (u32)M_WKC : 0u);
    clear = cs ? (cw ? (u32)(M_WKC | M_WQC) : (u32)(M_BKC | M_BQC)) : clear;
    s.meta = (s.meta & ~clear) ^ M_WHITE;  // current_player = other (lib.rs:778-780)
}

// ---- board-only key for 3-fold repetition (chess_v2.py:599-602) -------------------------
// A filter only: every hash hit is confirmed against the stored board, so collisions
// cannot change results.
GC_HD u64 mix64(u64 x) {
    x ^= x >> 31; x *= 0x7FB5D329728EA185ull;
    x ^= x >> 27; x *= 0x81DADEF4BC2DD44Dull;
    x ^= x >> 33;
    return x;
}
GC_HD u64 rotl64(u64 x, int r) { return (x << r) | (x >> (64 - r)); }
GC_HD u32 rotl32(u32 x, int r) { return (x << r) | (x >> (32 - r)); }
// The seven bitboards XORed, each rotated by its own amount (a move changes two squares of one
// or two boards), then the two halves mixed by one multiply each and a 32-bit finaliser: three
// 32-bit multiplies (the 64-bit multiply-sum it replaced took ~27 on the device, on the
// 3-fold role's critical phase).
GC_HD u32 board_key(const Pos& s) {
    const u64 x = s.k ^ rotl64(s.q, 11) ^ rotl64(s.r, 22) ^ rotl64(s.b, 37) ^ rotl64(s.n, 46) ^ rotl64(s.p, 55) ^
                  rotl64(s.w, 5);
    u32 y = ((u32)x * 0x9E3779B1u) ^ rotl32((u32)(x >> 32) * 0x85EBCA77u, 16);
    y ^= y >> 15;
    y *= 0x2C1B3C6Du;
    return y ^ (y >> 12);
}

// ---- mailbox <-> bitboards ------------------------------------------------------------
GC_HD Pos from_mailbox(const int8_t* b, u32 meta) {
    Pos s = {0, 0, 0, 0, 0, 0, 0, meta};
    for (int i = 0; i < 64; i++) put(s, i, b[i]);
    return s;
}
GC_HD void to_mailbox(const Pos& s, int8_t* b) {
    for (int i = 0; i < 64; i++) b[i] = (int8_t)id_at(s, i);
}

// ---- Philox4x32-10 random policy (same stream as the test oracle's policy draw) -----------
GC_HD u32 philox_x0(u64 seed, u32 board, u32 draw) {
    u32 k0 = (u32)seed, k1 = (u32)(seed >> 32);
    u32 x0 = board, x1 = draw, x2 = 0x5EEDu, x3 = 0u;
    // straight-line: a rolled loop here made the step kernels wait for every outstanding load
    // (the window probe in flight) at its header
#pragma unroll
    for (int i = 0; i < 10; i++) {
        u64 p0 = (u64)0xD2511F53u * x0;
        u64 p1 = (u64)0xCD9E8D57u * x2;
        u32 y0 = (u32)(p1 >> 32) ^ x1 ^ k0;
        u32 y1 = (u32)p1;
        u32 y2 = (u32)(p0 >> 32) ^ x3 ^ k1;
        u32 y3 = (u32)p0;
        x0 = y0; x1 = y1; x2 = y2; x3 = y3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return x0;
}
// uniform rank in [0, n) from the first Philox output word (multiply-shift)
GC_HD u32 scale_rank(u32 x0, u32 n) { return (u32)(((u64)x0 * n) >> 32); }
GC_HD u32 policy_index(u64 seed, u32 board, u32 draw, u32 n) { return scale_rank(philox_x0(seed, board, draw), n); }

}  // namespace gc
