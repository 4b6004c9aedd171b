// gc_env.h -- one ChessEnvV2.step() of the batched env, per lane.
//
// Restates /root/reference/gym_chess/envs/chess_v2.py:219-294 (opponent="none") on top
// of the bitboard core (gc_core.h), including the engine-call details the env relies on:
// State::new forcing of castle rights on every call (lib.rs:315-322), update_state after
// every next_state (lib.rs:1440), the "both kings checked" exception (lib.rs:1442-1446,
// reported here as reason R_BOTH_CHECKED with the state left unchanged), and the 3-fold
// repetition count keyed on the PRE-move board only (chess_v2.py:402-407, Q8).
//
// Repetition window.  A board can recur only between two irreversible moves: pawns never
// move backwards and no move adds a piece, so a pawn move or a capture strictly decreases
// a monotone potential and no later board equals an earlier one.  The window therefore
// holds the distinct boards since the last pawn move / capture (<= 300: the move cap,
// chess_v2.py:141, 252) with their occurrence counts.  Lookup is O(1): a per-board
// open-addressed table of 1024 entries {generation u32 | window slot u9 | key tag u22};
// an entry is live only if its generation equals the board's current one, so clearing
// the window (irreversible move, reset) is a single generation bump.  Every tag hit is
// confirmed against the stored 7-bitboard board, so the count is exact.
#pragma once
#include "gc_core.h"

namespace gc {

static constexpr int HIST_CAP = 300;
static constexpr int HTAB_BITS = 10;
static constexpr int HTAB = 1 << HTAB_BITS;
static constexpr int MOVES_MAX = 149;  // chess_v2.py:141

struct StepOut {
    int reward;
    int done;
    int reason;
    int moved;  // a move was applied (gen/ms describe the new position)
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

// H (per-board window storage) provides:
//   u32 gen(); void bump_gen();  u64 tab(int); void set_tab(int, u64);
//   bool same(int slot, const Pos&); void put(int slot, const Pos&);
//   int cnt(int slot); void set_cnt(int slot, int)
// Returns how many times the board has been the pre-move board so far, this one included.
template <class H>
GC_HD int rep_count(H& h, const Pos& s, u32& hl, bool irrev) {
    u32 key = board_key(s);
    u32 gen = h.gen();
    u32 pos = key & (HTAB - 1), tag = key >> HTAB_BITS;
    int c = 0;
    for (int probe = 0; probe < HTAB; probe++) {
        u64 e = h.tab(pos);
        if ((u32)e != gen) break;  // free for this generation
        if ((u32)(e >> 41) == tag) {
            int slot = (int)((e >> 32) & 511);
            if (h.same(slot, s)) {
                c = h.cnt(slot) + 1;
                h.set_cnt(slot, c);
                break;
            }
        }
        pos = (pos + 1) & (HTAB - 1);
    }
    if (irrev) {  // nothing before this move can recur: clear the window
        h.bump_gen();
        hl = 0;
        return c ? c : 1;
    }
    if (c) return c;
    if (hl < HIST_CAP) {
        h.put(hl, s);
        h.set_cnt(hl, 1);
        h.set_tab(pos, (u64)gen | ((u64)hl << 32) | ((u64)tag << 41));
        hl++;
    }
    return 1;
}

// One step().  On return with o.moved, `g`/`ms`/`scr` describe the new position (side now
// to move) so the caller can pick the next action without regenerating.  `g0` must be
// gen_init(s) when VALIDATE (external actions); the on-device policy is trusted.
template <bool VALIDATE, class H, class S>
GC_HD StepOut env_step(Pos& s, H& hist, int action, const Gen* g0, Gen& g, MoveSet& ms, S& scr) {
    StepOut o = {0, 0, R_NONE, 0};
    if (VALIDATE && !action_legal(s, *g0, action)) {  // chess_v2.py:240-242
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
    // update_state (lib.rs:1386-1393): the side now to move's flag comes from its own
    // generation pass; the mover's flag needs one attack probe.
    gen_init(ns, g);
    bool opp_chk = g.in_check;
    int mk = tracked_king(ns, white);
    bool my_chk = mk >= 0 && sq_attacked(ns, mk, !white);
    if (opp_chk && my_chk) {  // lib.rs:1442-1446
        o.reason = R_BOTH_CHECKED;
        o.done = 1;
        return o;
    }
    u32 chk = white ? ((my_chk ? M_WCHK : 0u) | (opp_chk ? M_BCHK : 0u))
                    : ((opp_chk ? M_WCHK : 0u) | (my_chk ? M_BCHK : 0u));
    u32 hl = hl_of(s.meta);
    bool rep = rep_count(hist, s, hl, irrev) >= 3;  // chess_v2.py:404-407
    ns.meta = with_hl((ns.meta & ~(u32)(M_WCHK | M_BCHK | M_DONE)) | chk | (rep ? M_DONE : 0u), hl);
    o.reward = -10 + mr;  // INVALID_ACTION_REWARD + move reward (Q9)
    o.moved = 1;
    if (rep) { o.done = 1; o.reason = R_REPETITION; }
    // the opponent's possible moves (chess_v2.py:268), mate (270-272), move_count (291-292)
    gen_moves(ns, g, ms, scr);
    if (ms.total == 0 && opp_chk) {
        ns.meta |= M_DONE;
        o.done = 1;
        o.reward += 100;
        o.reason = R_MATE;
    }
    if (!o.done && !white) ns.meta += (1u << M_MC_SHIFT);
    s = ns;
    return o;
}

}  // namespace gc
