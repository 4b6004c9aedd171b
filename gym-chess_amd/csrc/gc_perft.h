// gc_perft.h -- perft by composition of the reference's move generator and next_state
// (SURVEY.md §3.4): perft(s, d) = sum over get_all_possible_moves(s) of
// perft(next_state(s, m), d-1), perft(s, 1) = |moves|.  Every engine call re-reads the
// state dict, so State::new's rights forcing (lib.rs:315-322) applies to each child.
//
// One lane handles a subtree of depth <= 3 as two nested loops over the move lists (targets
// of the two interior levels parked in scratch slots, children picked in action-id order by
// the env policy's count-plane search -- any enumeration counts the same), with the last ply
// counted, not made ("bulk counting").  Deeper trees are split
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

template <class SA, class SB>
GC_HD uint64_t perft_small(const Pos& root, int depth, SA& sa, SB& sb) {
    if (depth <= 0) return 1;
    NoScratch none;
    Gen g0;
    MoveSet m0;
    gen_init(root, g0);
    if (depth == 1) {
        gen_moves(root, g0, m0, none);
        return (uint64_t)m0.total;
    }
    gen_moves(root, g0, m0, sa);
    uint64_t nodes = 0;
    for (int k1 = 0; k1 < m0.total; k1++) {
        Pos c1 = child_of(root, g0.white, select_action(root, g0, m0, sa, k1));
        Gen g1;
        MoveSet m1;
        gen_init(c1, g1);
        if (depth == 2) {
            gen_moves(c1, g1, m1, none);
            nodes += (uint64_t)m1.total;
            continue;
        }
        gen_moves(c1, g1, m1, sb);
        for (int k2 = 0; k2 < m1.total; k2++) {
            Pos c2 = child_of(c1, g1.white, select_action(c1, g1, m1, sb, k2));
            Gen g2;
            MoveSet m2;
            gen_init(c2, g2);
            gen_moves(c2, g2, m2, none);
            nodes += (uint64_t)m2.total;
        }
    }
    return nodes;
}

// perft_small at depth 2 only (one loop; one scratch for the root's parked targets): the
// split leaf level's kernel, small enough in registers for more waves per SIMD
template <class SA>
GC_HD uint64_t perft2(const Pos& root, SA& sa) {
    NoScratch none;
    Gen g0;
    MoveSet m0;
    gen_init(root, g0);
    gen_moves(root, g0, m0, sa);
    uint64_t nodes = 0;
    for (int k1 = 0; k1 < m0.total; k1++) {
        // any enumeration of the children counts the same: the action-id order pick of the
        // env policy (count planes, no per-piece walk) instead of the reference order
        Pos c1 = child_of(root, g0.white, select_action(root, g0, m0, sa, k1));
        Gen g1;
        MoveSet m1;
        gen_init(c1, g1);
        gen_moves(c1, g1, m1, none);
        nodes += (uint64_t)m1.total;
    }
    return nodes;
}

}  // namespace gc
