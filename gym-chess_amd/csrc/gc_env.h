// gc_env.h -- one ChessEnvV2.step() of the batched env, per lane.
//
// Restates /root/reference/gym_chess/envs/chess_v2.py:219-294 (opponent="none") on top
// of the bitboard core (gc_core.h), including the engine-call details the env relies on:
// State::new forcing of castle rights on every call (lib.rs:315-322), update_state after
// every next_state (lib.rs:1440), the "both kings checked" exception (lib.rs:1442-1446,
// reported here as reason R_BOTH_CHECKED with the state left unchanged), and the 3-fold
// repetition count keyed on the PRE-move board only (chess_v2.py:402-407, Q8).
//
// Repetition window: a board recurs only between two irreversible moves (pawn moves and
// captures strictly decrease a monotone potential -- pawns never move backwards and no
// move ever adds a piece), so the window is cleared on such moves.  It holds at most 300
// boards (the move cap, chess_v2.py:141, 252).  Keys are 32-bit board hashes; every key
// hit is confirmed against the stored 7-bitboard board, so the count is exact.
#pragma once
#include "gc_core.h"

namespace gc {

static constexpr int HIST_CAP = 300;
static constexpr int MOVES_MAX = 149;  // chess_v2.py:141

struct StepOut {
    int reward;
    int done;
    int reason;
    int moved;  // a move was applied: the caller must run env_finish() with the new list
};

GC_HD u32 mc_of(u32 meta) { return (meta & M_MC_MASK) >> M_MC_SHIFT; }
GC_HD u32 hl_of(u32 meta) { return (meta & M_HL_MASK) >> M_HL_SHIFT; }
GC_HD u32 with_hl(u32 meta, u32 hl) { return (meta & ~(u32)M_HL_MASK) | (hl << M_HL_SHIFT); }

// reset (chess_v2.py:183-206): board := initial, all four rights True then forced by
// State::new, check flags from update_state, WHITE to move, move_count 0, not done.
GC_HD Pos env_reset_pos(const Pos& init) {
    Pos s = init;
    s.meta = M_WHITE | M_RIGHTS;
    s.meta = (s.meta & ~(u32)M_RIGHTS) | eff_rights(s);
    s.meta |= check_flags(s);
    return s;
}

// H: repetition-window storage with
//   u32 key(int slot); bool same(int slot, const Pos&); void put(int slot, u32 key, const Pos&)
// `g` must be gen_init(s) when VALIDATE (external actions); trusted callers (the on-device
// policy picked `action` from this very state) skip the legality re-check.
template <bool VALIDATE, class H>
GC_HD StepOut env_step(Pos& s, H& hist, int action, const Gen* g) {
    StepOut o = {0, 0, R_NONE, 0};
    if (VALIDATE && !action_legal(s, *g, action)) {  // chess_v2.py:240-242
        o.reward = -10;
        o.done = (s.meta & M_DONE) ? 1 : 0;
        o.reason = R_INVALID;
        return o;
    }
    if (s.meta & M_DONE) { o.done = 1; o.reason = R_DONE_ALREADY; return o; }       // 245-251
    if (mc_of(s.meta) > MOVES_MAX) { o.done = 1; o.reason = R_MOVE_CAP; return o; }  // 252-258
    bool white = s.meta & M_WHITE;
    Pos ns = s;
    ns.meta = (ns.meta & ~(u32)M_RIGHTS) | eff_rights(s);  // State::new
    int mr;
    bool irrev;
    apply_move(ns, white, action, &mr, &irrev);
    u32 chk = check_flags(ns);
    if ((chk & (M_WCHK | M_BCHK)) == (M_WCHK | M_BCHK)) {  // lib.rs:1442-1446
        o.reason = R_BOTH_CHECKED;
        o.done = 1;
        return o;
    }
    // 3-fold on the pre-move board (chess_v2.py:404-407)
    u32 hl = hl_of(s.meta);
    u32 key = board_key(s);
    int cnt = 1;
    for (u32 i = 0; i < hl; i++)
        if (hist.key(i) == key && hist.same(i, s)) cnt++;
    bool rep = cnt >= 3;
    if (irrev) hl = 0;
    else if (hl < HIST_CAP) { hist.put(hl, key, s); hl++; }
    ns.meta = with_hl((ns.meta & ~(u32)(M_WCHK | M_BCHK | M_DONE)) | chk | (rep ? M_DONE : 0u), hl);
    o.reward = -10 + mr;  // INVALID_ACTION_REWARD + move reward (Q9)
    o.moved = 1;
    if (rep) { o.done = 1; o.reason = R_REPETITION; }
    s = ns;
    return o;
}

// The part of step() after the opponent's move list is known (chess_v2.py:268-292):
// mate bonus, done, move_count.  `n_next` = legal move count of the side now to move.
GC_HD void env_finish(Pos& s, StepOut& o, int n_next) {
    bool wtm = s.meta & M_WHITE;
    bool opp_chk = wtm ? (s.meta & M_WCHK) : (s.meta & M_BCHK);
    if (n_next == 0 && opp_chk) {  // 270-272
        s.meta |= M_DONE;
        o.done = 1;
        o.reward += 100;
        o.reason = R_MATE;
    }
    if (o.done) return;                                     // 273-274
    if (wtm) s.meta += (1u << M_MC_SHIFT);                  // 291-292
}

}  // namespace gc
