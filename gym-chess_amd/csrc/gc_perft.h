// gc_perft.h -- perft by composition of the reference's move generator and next_state
// (SURVEY.md §3.4): perft(s, d) = sum over get_all_possible_moves(s) of
// perft(next_state(s, m), d-1), perft(s, 1) = |moves|.  Every engine call re-reads the
// state dict, so State::new's rights forcing (lib.rs:315-322) applies to each child.
//
// One lane handles a subtree of depth <= 3 as two nested loops over the move lists (targets
// of the two interior levels parked in scratch slots), with the last ply
// counted, not made ("bulk counting").  Children are enumerated by walking the parked
// targets (MoveWalk), not by rank.  Deeper trees are split
// into such subtrees by expanding whole levels on the device (gymchess.hip).
#pragma once
#include "gc_core.h"

namespace gc {

GC_HD Pos child_of(const Pos& s, bool white, int action) {
    Pos c = s;
    int rw;
    bool irrev;
    apply_legal(c, white, action, &rw, &irrev);  // a generated (legal) move: the branch-free path
    c.meta = (c.meta & ~(u32)M_RIGHTS) | eff_rights(c);
    return c;
}

// Walks the legal moves gen_moves parked (!ms.big): own pieces in square order, each
// piece's targets low to high (fast pawns from their origin sets), then the castles.  Any
// enumeration counts the same; a step is a ctz and a mask (and, on a piece change, one
// slot read) where select_action's rank search is ~10x that.
struct MoveWalk {
    u64 pcs, tg;
    int sq, j;
    u32 castles;
    GC_HDM explicit MoveWalk(const Gen& g) : pcs(g.own), tg(0), sq(0), j(-1), castles(g.castles) {}
    template <class S>
    GC_HDM int next(const Gen& g, const MoveSet& ms, const S& scr) {
        while (tg == 0 && pcs) {
            sq = ctz(pcs);
            pcs &= pcs - 1;
            j++;
            tg = ((ms.fastp >> sq) & 1) ? fast_pawn_targets(ms, sq, g.white) : scr.get(j);
        }
        if (tg) {
            int t = ctz(tg);
            tg &= tg - 1;
            return sq * 64 + t;
        }
        if (castles & 1) {
            castles &= ~1u;
            return g.white ? A_QSW : A_QSB;
        }
        castles &= ~2u;
        return g.white ? A_KSW : A_KSB;
    }
};

// the k-th child's action: the walk, or the rank search when the position has more pieces
// than scratch slots (nothing parked)
template <class S>
GC_HD int next_child(MoveWalk& w, const Pos& s, const Gen& g, const MoveSet& ms, const S& scr, int k) {
    return ms.big ? select_action(s, g, ms, scr, k) : w.next(g, ms, scr);
}

template <class SA, class SB>
GC_HD uint64_t perft_small(const Pos& root, int depth, SA& sa, SB& sb) {
    if (depth <= 0) return 1;
    Gen g0;
    MoveSet m0;
    gen_init(root, g0);
    if (depth == 1) return (uint64_t)count_moves(root, g0);
    gen_moves(root, g0, m0, sa);
    uint64_t nodes = 0;
    MoveWalk w0(g0);
    // the children's side to move is the other side, whose king the root's moves leave in place
    const KingLines k1l = king_lines_of(root, !g0.white);
    for (int k1 = 0; k1 < m0.total; k1++) {
        Pos c1 = child_of(root, g0.white, next_child(w0, root, g0, m0, sa, k1));
        if (depth == 2) {
            nodes += (uint64_t)count_position_kl(c1, k1l);
            continue;
        }
        Gen g1;
        MoveSet m1;
        gen_init(c1, g1);
        gen_moves(c1, g1, m1, sb);
        MoveWalk w1(g1);
        const KingLines k2l = king_lines_of(c1, !g1.white);
        for (int k2 = 0; k2 < m1.total; k2++) {
            Pos c2 = child_of(c1, g1.white, next_child(w1, c1, g1, m1, sb, k2));
            nodes += (uint64_t)count_position_kl(c2, k2l);
        }
    }
    return nodes;
}

// perft_small at depth 2 only (one loop; one scratch for the root's parked targets): the
// split leaf level's kernel, small enough in registers for more waves per SIMD
template <class SA>
GC_HD uint64_t perft2(const Pos& root, SA& sa, const u64* ntab = nullptr) {
    Gen g0;
    MoveSet m0;
    gen_init(root, g0);
    gen_moves(root, g0, m0, sa);
    uint64_t nodes = 0;
    const KingLines k1l = king_lines_of(root, !g0.white);  // as perft_small
    if (m0.big) {  // more pieces than scratch slots (rare): children by rank
        for (int k1 = 0; k1 < m0.total; k1++)
            nodes += (uint64_t)count_position_kl(child_of(root, g0.white, select_action(root, g0, m0, sa, k1)), k1l);
        return nodes;
    }
    // the walk alone (its own loop: the context and count planes the rank search would need are
    // dead here, which keeps the loop's live registers down)
    MoveWalk w0(g0);
    for (int k1 = 0; k1 < m0.total; k1++) {
        Pos c1 = child_of(root, g0.white, w0.next(g0, m0, sa));
        nodes += (uint64_t)count_position_kl(c1, k1l, ntab);
    }
    return nodes;
}

}  // namespace gc
