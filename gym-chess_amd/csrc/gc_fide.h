// gc_fide.h -- optional FIDE rules for the engine and the env.
//
// OUTSIDE the reference-parity contract: the reference plays its own rules (gc_core.h,
// SURVEY §0 Q1-Q10).  rules = FIDE changes exactly what §8f row 4 names:
//   * en passant (target square in the meta word; generated only when legal, the
//     horizontal discovered check included);
//   * real promotion: perft counts all four pieces; env actions (from*64+to, no piece
//     field in the reference's 4101-action space) promote to a queen, with the reference's
//     +10 promotion reward (lib.rs:700-709);
//   * castling: per-side rights (K for king side, Q for queen side, not their OR), king and
//     rook of the mover's colour on their squares (black castles with black pieces), the
//     king not in check and not crossing or landing on an attacked square; rights revoked
//     by any king move, a rook leaving its corner or a capture on that corner;
//   * pawns' double step needs both squares empty; kings are never captured and never
//     retreat along a checking ray (the enemy map is built with the own king removed).
// Everything else is the reference env's: rewards (-10 per valid move + capture value,
// +-100 on mate), the move cap, 3-fold on the board alone, the random-policy driver.
// Validated against published perft counts (tests/test_fide.py).
//
// Same square numbering and piece ids as gc_core.h; meta bits 25..28 hold en passant.
#pragma once
#include "gc_core.h"
#include "gc_env.h"

namespace gc {
namespace fide {

enum : u32 { M_EP = 1u << 25, M_EP_SHIFT = 26, M_EP_MASK = 7u << 26 };
static constexpr u64 ROW0 = 0xFFull;        // rank 8: white promotes here
static constexpr u64 ROW7 = 0xFFull << 56;  // rank 1: black promotes here

// en passant target (the square a capturing pawn lands on) or -1
GC_HD int ep_square(u32 meta) {
    int file = (int)((meta & M_EP_MASK) >> M_EP_SHIFT);
    int sq = (meta & M_WHITE) ? 16 + file : 40 + file;
    return (meta & M_EP) ? sq : -1;
}
GC_HD u32 with_ep(u32 meta, int file) {  // file < 0: none
    meta &= ~(u32)(M_EP | M_EP_MASK);
    return file < 0 ? meta : (meta | M_EP | ((u32)file << M_EP_SHIFT));
}

struct FGen {
    Gen g;        // side, occupancy, king, check mask, pins, enemy map (own king removed), castles
    u64 ep_from;  // own pawns with a LEGAL en-passant capture onto g_ep
    int ep;       // en-passant target square, or -1
};

// is the king on ks attacked by the enemy pieces in `opp`, given the occupancy `occ`?
// (en-passant legality: both are the position after the capture)
GC_HD bool king_hit(const Pos& s, int ks, bool white, u64 occ, u64 opp) {
    u64 kb = bit(ks);
    u64 att = (rook_att(ks, occ) & (s.r | s.q) & opp) | (bishop_att(ks, occ) & (s.b | s.q) & opp) |
              (knight_set(kb) & s.n & opp) | (pawn_att_set(kb, white) & s.p & opp) | (king_set(kb) & s.k & opp);
    return att != 0;
}

GC_HD void fgen(const Pos& s, FGen& f) {
    Gen& g = f.g;
    gen_base(s, g);
    f.ep = -1;
    f.ep_from = 0;
    u64 myk = s.k & g.own;
    g.ks = myk ? ctz(myk) : -1;  // FIDE positions hold one king per side
    gen_pins(s, g);              // checkers / check mask / pin segments: rules-neutral
    bool white = g.white;
    if (g.ks >= 0) {
        Pos t = s;  // enemy map with the own king removed: no retreat along a checking ray
        t.k &= ~myk;
        t.w &= ~myk;
        g.enemy_att = side_attacks(t, !white);
        int base = white ? 56 : 0;
        bool kok = (myk & bit(base + 4)) && !g.in_check;
        u64 myr = s.r & g.own, A = g.enemy_att, occ = g.occ;
        bool ksr = (s.meta & (white ? M_WKC : M_BKC)) != 0, qsr = (s.meta & (white ? M_WQC : M_BQC)) != 0;
        bool kside = kok && ksr && (myr & bit(base + 7)) && !(occ & (3ull << (base + 5))) && !(A & (3ull << (base + 5)));
        bool qside = kok && qsr && (myr & bit(base)) && !(occ & (7ull << (base + 1))) && !(A & (3ull << (base + 2)));
        g.castles = (qside ? 1u : 0u) | (kside ? 2u : 0u);
    }
    int ept = ep_square(s.meta);
    if (ept >= 0) {
        int cap = white ? ept + 8 : ept - 8;  // the pawn that just stepped twice
        u64 cand = pawn_att_set(bit(ept), !white) & s.p & g.own;
        bool ok = (s.p & g.opp & bit(cap)) && !(g.occ & bit(ept));
        while (ok && cand) {
            int fr = ctz(cand);
            cand &= cand - 1;
            u64 occ2 = (g.occ ^ bit(fr) ^ bit(cap)) | bit(ept);
            if (g.ks < 0 || !king_hit(s, g.ks, white, occ2, g.opp & ~bit(cap))) f.ep_from |= bit(fr);
        }
        if (f.ep_from) f.ep = ept;
    }
}

// legal targets of the own piece on sq (type t): promotions once (the to-square), en passant
// included for pawns.  Enemy kings are never targets.
GC_HD u64 ftargets(const Pos& s, const FGen& f, int sq, int t) {
    const Gen& g = f.g;
    u64 m = bit(sq), notown = ~g.own & ~(s.k & g.opp);
    if (t == KING) return king_set(m) & notown & ~g.enemy_att;
    u64 tg;
    switch (t) {
        case QUEEN: tg = rook_att(sq, g.occ) | bishop_att(sq, g.occ); break;
        case ROOK: tg = rook_att(sq, g.occ); break;
        case BISHOP: tg = bishop_att(sq, g.occ); break;
        case KNIGHT: tg = knight_set(m); break;
        default: {  // PAWN: one step, two steps over an empty square, diagonal captures
            u64 empty = ~g.occ;
            u64 one = g.white ? ((m >> 8) & empty) : ((m << 8) & empty);
            u64 two = g.white ? (((one & (0xFFull << 40)) >> 8) & empty) : (((one & (0xFFull << 16)) << 8) & empty);
            tg = one | two | (pawn_att_set(m, g.white) & g.opp);
        }
    }
    tg &= notown;
    if (g.ks >= 0) {
        tg &= g.checkmask;
        if (g.pinned & m) tg &= g.pinrays & line_through(g.ks, sq);
    }
    if (t == PAWN && (f.ep_from & m)) tg |= bit(f.ep);  // legality tested in fgen
    return tg;
}

GC_HD u64 promo_row(bool white) { return white ? ROW0 : ROW7; }

// The shared type-uniform generator (gc_core.h gen_moves_a/b with F = true: pawns set-wise,
// one loop per piece type, targets parked per ordinal, bit-sliced count planes) for FIDE
// positions with at most SCRATCH_SLOTS own pieces; the per-square walk below serves the rest.
template <class S>
GC_HD void fgen_moves(const Pos& s, const FGen& f, MoveSet& ms, S& scr) {
    moveset_clear(ms);
    FideExtra fx{f.ep_from, f.ep};
    int total = popc(f.g.castles);
    total += gen_moves_a<S, true>(s, f.g, ms, scr, fx);
    total += gen_moves_b<S, true>(s, f.g, ms, scr);
    ms.total = total;
}
GC_HD bool fuses_walk(const FGen& f) { return popc(f.g.own) > SCRATCH_SLOTS; }

// number of legal moves, promotions counted once (env actions) or four times (perft):
// per-square walk (> SCRATCH_SLOTS own pieces)
GC_HD int fcount_walk(const Pos& s, const FGen& f, bool perft) {
    int n = popc(f.g.castles);
    u64 pcs = f.g.own;
    while (pcs) {
        int sq = ctz(pcs);
        pcs &= pcs - 1;
        int t = type_at(s, sq);
        u64 tg = ftargets(s, f, sq, t);
        n += popc(tg);
        if (perft && t == PAWN) n += 3 * popc(tg & promo_row(f.g.white));
    }
    return n;
}

// the same count through the shared generator
GC_HD int fcount(const Pos& s, const FGen& f, bool perft) {
    if (fuses_walk(f)) return fcount_walk(s, f, perft);
    MoveSet ms;
    NoScratch none;
    fgen_moves(s, f, ms, none);
    int n = ms.total;
    if (perft) {  // three more per promoting move (the origins on the last-but-one rank)
        u64 pre = f.g.white ? (0xFFull << 8) : (0xFFull << 48);
        n += 3 * (popc(ms.o1 & pre) + popc(ms.ol & pre) + popc(ms.orr & pre));  // per move, not per pawn
        FideExtra fx{f.ep_from, f.ep};
        u64 pp = s.p & f.g.own & f.g.pinned & pre;
        while (pp) {
            int sq = ctz(pp);
            pp &= pp - 1;
            n += 3 * popc(fide_pawn_targets(s, f.g, sq, fx) & promo_row(f.g.white));
        }
    }
    return n;
}

// k-th legal ACTION in ascending action id (from*64+to, then castles: king side 4096/4098
// before queen side 4097/4099) -- the random policy's order, as in the reference mode
GC_HD int fselect(const Pos& s, const FGen& f, int k) {
    u64 pcs = f.g.own;
    while (pcs) {
        int sq = ctz(pcs);
        pcs &= pcs - 1;
        u64 tg = ftargets(s, f, sq, type_at(s, sq));
        int c = popc(tg);
        if (k < c) return sq * 64 + kth_set_bit(tg, k);
        k -= c;
    }
    bool w = f.g.white;
    if (f.g.castles & 2) { if (k == 0) return w ? A_KSW : A_KSB; k--; }
    if (f.g.castles & 1) { if (k == 0) return w ? A_QSW : A_QSB; }
    return A_NONE;
}

// Set-wise generation under FIDE rules (gc_core.h sw_*, the self-play policy's move-set
// order): the double step needs the square between empty, enemy kings are never targets, and
// the legal en-passant captures (ep_from, legality from fgen) join the capture sets.
GC_HD void fsw_pawns(const Pos& s, const FGen& f, u64* t) {
    const Gen& g = f.g;
    const u64 cm = g.checkmask, empty = ~g.occ, opp = g.opp & ~s.k, P = s.p & g.own, pr = g.pinrays;
    const int kq = sw_ksq(g);
    const u64 fp = P & ~g.pinned, pp = P & g.pinned;
    const u64 pf = pp & file_mask(kq), pd = pp & diag_mask(kq), pa = pp & anti_mask(kq);
    const u64 epb = f.ep >= 0 ? bit(f.ep) : 0ull, ef = f.ep_from;
    if (g.white) {
        const u64 mf = ((fp & ROW6) >> 8) & empty, mp = ((pf & ROW6) >> 8) & empty;
        t[SW_P1] = ((fp >> 8) | ((pf >> 8) & pr)) & empty & cm;
        t[SW_P2] = ((mf >> 8) | ((mp >> 8) & pr)) & empty & cm;
        t[SW_PL] = ((((fp >> 7) | ((pa >> 7) & pr)) & ~FILE_A) & opp & cm) | (((ef >> 7) & ~FILE_A) & epb);
        t[SW_PR] = ((((fp >> 9) | ((pd >> 9) & pr)) & ~FILE_H) & opp & cm) | (((ef >> 9) & ~FILE_H) & epb);
    } else {
        const u64 mf = ((fp & ROW1) << 8) & empty, mp = ((pf & ROW1) << 8) & empty;
        t[SW_P1] = ((fp << 8) | ((pf << 8) & pr)) & empty & cm;
        t[SW_P2] = ((mf << 8) | ((mp << 8) & pr)) & empty & cm;
        t[SW_PL] = ((((fp << 9) | ((pd << 9) & pr)) & ~FILE_A) & opp & cm) | (((ef << 9) & ~FILE_A) & epb);
        t[SW_PR] = ((((fp << 7) | ((pa << 7) & pr)) & ~FILE_H) & opp & cm) | (((ef << 7) & ~FILE_H) & epb);
    }
}
// the sets of part A (pawns, knights, kings) and B (sliders), as the paired kernel splits them
GC_HD void fsw_gen_a(const Pos& s, const FGen& f, u64* t) {
    const u64 nk = ~(s.k & f.g.opp);
    fsw_pawns(s, f, t);
    sw_knights(s, f.g, t, nk);
    sw_kings(s, f.g, t, nk);
}
GC_HD void fsw_gen_b(const Pos& s, const FGen& f, u64* t) {
    const u64 nk = ~(s.k & f.g.opp);
    sw_orth(s, f.g, t, nk);
    sw_diag(s, f.g, t, nk);
}
GC_HD int fsw_gen(const Pos& s, const FGen& f, u64* t) {
    fsw_gen_a(s, f, t);
    fsw_gen_b(s, f, t);
    return sw_popc(t, 0, SW_SETS) + popc(f.g.castles);
}

// the random policy's pick for the side to move of s (fgen'd into f): draws k uniformly in
// [0, #legal) from the Philox stream (board, draw++) and returns the k-th legal action in
// move-set order (as the reference-rules self-play)
template <class S>
GC_HD int fpick_action(const Pos& s, const FGen& f, S&, uint64_t seed, u32 board, u32& draw) {
    u64 t[SW_SETS];
    const int n = fsw_gen(s, f, t);
    if (n == 0) return A_NONE;
    return sw_select(f.g, t, (int)policy_index(seed, board, draw++, (u32)n));
}

GC_HD bool faction_legal(const Pos& s, const FGen& f, int action) {
    if (action < 0 || action > A_RESIGN) return false;
    bool w = f.g.white;
    if (action >= 4096) {
        if (w) return (action == A_QSW && (f.g.castles & 1)) || (action == A_KSW && (f.g.castles & 2));
        return (action == A_QSB && (f.g.castles & 1)) || (action == A_KSB && (f.g.castles & 2));
    }
    int fr = action >> 6, to = action & 63;
    if (!((f.g.own >> fr) & 1)) return false;
    return (ftargets(s, f, fr, type_at(s, fr)) >> to) & 1;
}

// castling rights lost when a move touches a square (from or to): the kings' and rooks'
// start squares (a8 = 0, e8 = 4, h8 = 7, a1 = 56, e1 = 60, h1 = 63)
GC_HD u32 rights_lost(int sq) {
    u32 r = 0;
    r |= sq == 0 ? (u32)M_BQC : 0u;
    r |= sq == 7 ? (u32)M_BKC : 0u;
    r |= sq == 4 ? (u32)(M_BKC | M_BQC) : 0u;
    r |= sq == 56 ? (u32)M_WQC : 0u;
    r |= sq == 63 ? (u32)M_WKC : 0u;
    r |= sq == 60 ? (u32)(M_WKC | M_WQC) : 0u;
    return r;
}

// apply a move of the side to move.  action: from*64+to or a castle id; promo: piece type
// for a pawn reaching the last rank (0 = queen).  Returns -1 if the from-square holds no
// piece of the side to move, -2 for an action id that is no move.  *reward = captured value
// (+10 for a promotion: lib.rs:700-709), *irrev = pawn move or capture.
GC_HD int fapply(Pos& s, int action, int promo, int* reward, bool* irrev) {
    bool white = s.meta & M_WHITE;
    *reward = 0;
    *irrev = false;
    u64 own = white ? s.w : (occ_of(s) & ~s.w);
    if (action >= 4096) {
        int kf, kt, rf, rt;
        switch (action) {
            case A_KSW: kf = 60; kt = 62; rf = 63; rt = 61; break;
            case A_QSW: kf = 60; kt = 58; rf = 56; rt = 59; break;
            case A_KSB: kf = 4; kt = 6; rf = 7; rt = 5; break;
            case A_QSB: kf = 4; kt = 2; rf = 0; rt = 3; break;
            default: return -2;
        }
        int sgn = white ? 1 : -1;
        clear_sq(s, kf); clear_sq(s, rf);
        put(s, kt, KING * sgn); put(s, rt, ROOK * sgn);
        s.meta &= white ? ~(u32)(M_WKC | M_WQC) : ~(u32)(M_BKC | M_BQC);
        s.meta = with_ep(s.meta, -1) ^ M_WHITE;
        return 0;
    }
    int fr = action >> 6, to = action & 63;
    if (!((own >> fr) & 1)) return -1;
    int pt = type_at(s, fr);
    int ept = ep_square(s.meta);
    int cap_sq = to, ct;
    if (pt == PAWN && to == ept && ((fr ^ to) & 7)) {  // en passant
        cap_sq = white ? to + 8 : to - 8;
        ct = PAWN;
    } else {
        ct = type_at(s, to);
    }
    *reward = (int)((0x1335A00u >> (4 * ct)) & 0xFu);  // lib.rs:19-25 values by |id|
    *irrev = pt == PAWN || ct != EMPTY;
    clear_sq(s, fr);
    clear_sq(s, cap_sq);
    int nt = pt;
    if (pt == PAWN && (bit(to) & promo_row(white))) {
        nt = promo ? promo : QUEEN;
        *reward += 10;
    }
    put(s, to, white ? nt : -nt);
    s.meta &= ~(rights_lost(fr) | rights_lost(to));
    int dbl = pt == PAWN && (fr - to == 16 || to - fr == 16);
    s.meta = with_ep(s.meta, dbl ? (fr & 7) : -1) ^ M_WHITE;
    return 0;
}

// both check flags (update_state) under FIDE rules: king attacked by the other side
GC_HD u32 fcheck_flags(const Pos& s) {
    u64 occ = occ_of(s);
    u32 fl = 0;
    u64 wk = s.k & s.w, bk = s.k & occ & ~s.w;
    if (wk && king_hit(s, ctz(wk), true, occ, occ & ~s.w)) fl |= M_WCHK;
    if (bk && king_hit(s, ctz(bk), false, occ, s.w)) fl |= M_BCHK;
    return fl;
}

// perft by explicit enumeration (promotions x4), depth <= 3 per lane; leaves bulk-counted
template <int D>
GC_HD uint64_t fperft(const Pos& s) {
    FGen f;
    fgen(s, f);
    if constexpr (D <= 1) {
        return (uint64_t)fcount(s, f, true);
    } else {
        uint64_t n = 0;
        u64 pcs = f.g.own;
        while (pcs) {
            int sq = ctz(pcs);
            pcs &= pcs - 1;
            int t = type_at(s, sq);
            u64 tg = ftargets(s, f, sq, t);
            while (tg) {
                int to = ctz(tg);
                tg &= tg - 1;
                int np = (t == PAWN && (bit(to) & promo_row(f.g.white))) ? 4 : 1;
                for (int pc = 0; pc < np; pc++) {
                    Pos c = s;
                    int rw;
                    bool irr;
                    fapply(c, sq * 64 + to, np == 4 ? QUEEN + pc : 0, &rw, &irr);
                    n += fperft<D - 1>(c);
                }
            }
        }
        for (int cb = 0; cb < 2; cb++) {
            if (!(f.g.castles & (1u << cb))) continue;
            Pos c = s;
            int rw;
            bool irr;
            fapply(c, cb ? (f.g.white ? A_KSW : A_KSB) : (f.g.white ? A_QSW : A_QSB), 0, &rw, &irr);
            n += fperft<D - 1>(c);
        }
        return n;
    }
}
GC_HD uint64_t fperft_small(const Pos& s, int depth) {
    if (depth <= 0) return 1;
    if (depth == 1) return fperft<1>(s);
    if (depth == 2) return fperft<2>(s);
    return fperft<3>(s);
}

// ---- env step under FIDE rules (chess_v2.py:219-294 with the moves above) -----------------
// Same contract as gc_env.h env_step: on o.moved, `f` describes the new position.
template <bool VALIDATE, class H>
GC_HD StepOut fenv_step(Pos& s, H& hist, int action, FGen& f) {
    StepOut o = {0, 0, R_NONE, 0};
    if (VALIDATE) {
        FGen f0;
        fgen(s, f0);
        if (!faction_legal(s, f0, action)) {
            o.reward = -10;
            o.done = (s.meta & M_DONE) ? 1 : 0;
            o.reason = R_INVALID;
            return o;
        }
    }
    if (s.meta & M_DONE) { o.done = 1; o.reason = R_DONE_ALREADY; return o; }
    if (mc_of(s.meta) > MOVES_MAX) { o.done = 1; o.reason = R_MOVE_CAP; return o; }
    bool white = s.meta & M_WHITE;
    RepProbe pr;
    rep_prefetch(hist, s, pr);
    Pos ns = s;
    int mr;
    bool irrev;
    fapply(ns, action, 0, &mr, &irrev);
    u32 chk = fcheck_flags(ns);
    fgen(ns, f);
    u32 hl = hl_of(s.meta);
    int c = rep_commit(hist, s, pr, hl, irrev);
    bool rep = c >= 3;
    ns.meta = with_hl((ns.meta & ~(u32)(M_WCHK | M_BCHK | M_DONE)) | chk | ((rep || c == 0) ? M_DONE : 0u), hl);
    s = ns;
    o.reward = -10 + mr;
    o.moved = 1;
    if (rep) { o.done = 1; o.reason = R_REPETITION; }
    if (c == 0) { o.done = 1; o.reason = R_WINDOW_FULL; }
    if (f.g.in_check && fcount(s, f, false) == 0) {  // mate
        s.meta |= M_DONE;
        o.done = 1;
        o.reward += 100;
        o.reason = R_MATE;
    }
    if (!o.done && !white) s.meta += (1u << M_MC_SHIFT);
    return o;
}

// ---- the random opponent under FIDE rules (chess_v2.py:219-294 with opponent_policy set;
// the reference-rules env_step_vs / env_open_vs of gc_env.h with the moves above) -----------
// one ply of the env: `action` (legal) from s; the window commit, the new position's `f`,
// the move reward and the 3-fold count (c >= 3: repetition, 0: window full)
template <class H>
GC_HD void fenv_ply(Pos& s, H& hist, int action, FGen& f, int* mr, int* c) {
    RepProbe pr;
    rep_prefetch(hist, s, pr);
    Pos ns = s;
    bool irrev;
    fapply(ns, action, 0, mr, &irrev);
    const u32 chk = fcheck_flags(ns);
    fgen(ns, f);
    u32 hl = hl_of(s.meta);
    *c = rep_commit(hist, s, pr, hl, irrev);
    ns.meta = with_hl((ns.meta & ~(u32)(M_WCHK | M_BCHK | M_DONE)) | chk | ((*c >= 3 || *c == 0) ? M_DONE : 0u), hl);
    s = ns;
}
// the agent's (validated) action, then -- unless that ended the episode -- the opponent's
// reply drawn from the policy stream (fpick_action: one draw); on o.moved `f` describes the
// final position
template <bool VALIDATE, class H, class S>
GC_HD StepOut fenv_step_vs(Pos& s, H& hist, int action, FGen& f, S& scr, uint64_t seed, u32 board, u32& draw) {
    StepOut o = {0, 0, R_NONE, 0};
    if (VALIDATE) {
        FGen f0;
        fgen(s, f0);
        if (!faction_legal(s, f0, action)) {
            o.reward = -10;
            o.done = (s.meta & M_DONE) ? 1 : 0;
            o.reason = R_INVALID;
            return o;
        }
    }
    if (s.meta & M_DONE) { o.done = 1; o.reason = R_DONE_ALREADY; return o; }
    if (mc_of(s.meta) > MOVES_MAX) { o.done = 1; o.reason = R_MOVE_CAP; return o; }
    int mr, c;
    fenv_ply(s, hist, action, f, &mr, &c);
    o.reward = -10 + mr;
    o.moved = 1;
    if (c >= 3) { o.done = 1; o.reason = R_REPETITION; }
    if (c == 0) { o.done = 1; o.reason = R_WINDOW_FULL; }
    const int n = fcount(s, f, false);
    if (f.g.in_check && n == 0) {  // 270-272
        s.meta |= M_DONE;
        o.done = 1;
        o.reward += 100;
        o.reason = R_MATE;
    }
    if (o.done) return o;
    if (n == 0) {  // 120-122: the opponent has no move ("resign")
        s.meta |= M_DONE;
        o.done = 1;
        o.reason = R_OPP_NO_MOVE;
        return o;
    }
    hist.commit();  // the agent ply's window write lands before the reply probes it
    const int oa = fpick_action(s, f, scr, seed, board, draw);
    fenv_ply(s, hist, oa, f, &mr, &c);
    o.reward -= mr;  // 283
    if (c >= 3) { o.done = 1; o.reason = R_REPETITION; }
    if (c == 0) { o.done = 1; o.reason = R_WINDOW_FULL; }
    if (f.g.in_check && fcount(s, f, false) == 0) {  // 285-288
        s.meta |= M_DONE;
        o.done = 1;
        o.reward -= 100;
        o.reason = R_MATED;
    }
    if (s.meta & M_WHITE) s.meta += (1u << M_MC_SHIFT);  // 291-292
    return o;
}
// reset() for a BLACK agent (chess_v2.py:208-216): the opponent opens from the reset
// position (WHITE to move, `f` its generation); its 3-fold verdict is discarded and
// move_count becomes 1; with no opening move the env is left done.  `f` then describes the
// agent's position.
template <class H, class S>
GC_HD void fenv_open_vs(Pos& s, H& hist, FGen& f, S& scr, uint64_t seed, u32 board, u32& draw) {
    if (fcount(s, f, false) == 0) { s.meta |= M_DONE; return; }
    const int oa = fpick_action(s, f, scr, seed, board, draw);
    int mr, c;
    fenv_ply(s, hist, oa, f, &mr, &c);
    s.meta = (s.meta & ~(u32)M_DONE) + (1u << M_MC_SHIFT);
}

}  // namespace fide
}  // namespace gc
