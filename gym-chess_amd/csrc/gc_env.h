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
// chess_v2.py:141, 252) with their occurrence counts, in a per-board open-addressed table
// of HTAB 64-byte entries {generation u32 | key tag u23 | count u8, 7 bitboards}: one
// entry = one cache line, so a single probe both finds and verifies a board.  An entry is
// live only if its generation equals the board's current one, so clearing the window
// (irreversible move, reset) is a single generation bump.  The count is exact (full-board
// compare); the first probe is issued before move generation so its latency overlaps it.
#pragma once
#include "gc_core.h"

#ifndef GC_STAMP
#define GC_STAMP(k)  // diagnostic builds (-DGC_STAMPS) record s_memtime at phase boundaries
#endif

namespace gc {

// Window capacity.  With opponent "none" (and a WHITE agent) the move cap bounds a window to
// ~301 boards; a BLACK agent's move_count never advances (chess_v2.py:291-292), so its
// window is unbounded in the reference (saved_boards grows for the whole game,
// chess_v2.py:192, 404-407).  The per-board table size is per env (H::bits()):
//  * 2^9 = 512 entries (32 KiB per board, 2 GiB at 65 536 boards) when the move cap bounds
//    the games (opponent "none", or a WHITE agent): windows of <= ~301 boards, load <= 0.59;
//    a window may hold HIST_CAP = 384 boards there (load 0.75);
//  * 2^10 = 1024 entries for a BLACK agent, whose games have no move cap: the table holds
//    511 boards of a window (the 9-bit window-length field of the meta word, load 0.5), and
//    every further board of that window goes to the env's SPILL table (below), so no window
//    length ends an episode.  R_WINDOW_FULL now means only that the spill table itself ran
//    out of probes -- the host grows it long before (gc_env_*), and reports the error.
static constexpr int HTAB_BITS = 9;                 // the move-capped envs (all paired kernels)
static constexpr int HTAB_BITS_UNCAPPED = 10;       // BLACK agent
static constexpr int HTAB = 1 << HTAB_BITS;
static constexpr int HTAB_MAX = 1 << HTAB_BITS_UNCAPPED;
GC_HD int hist_cap(int bits) { return bits > HTAB_BITS ? 511 : 384; }
GC_HD u32 tag_mask(int bits) { return (1u << (32 - bits)) - 1; }  // key bits above the slot index
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

// one table entry
struct RepEntry {
    u64 hdr;  // gen (bits 0..31) | tag (32.., 32 - bits wide) | count (56..63)
    u64 k, q, r, b, n, p, w;
};
GC_HD bool rep_same(const RepEntry& e, const Pos& s) {
    return e.k == s.k && e.q == s.q && e.r == s.r && e.b == s.b && e.n == s.n && e.p == s.p && e.w == s.w;
}

// H (per-board table storage) provides:
//   int bits(); u32 gen(); void bump_gen(); RepEntry load(int pos); void store_hdr(int pos, u64);
//   void store(int pos, const RepEntry&)
// and the spill table (one per env, shared by its boards; only for a BLACK agent's windows
// past hist_cap, whose table is full -- hl saturates at hist_cap while a window spills):
//   u32 spill_mask() (0: no spill table), u32 owner() (the board), u64 sp_hdr(u32 slot)
//   (coherent load), bool sp_cas(u32 slot, u64& expect, u64 desired) (device-wide; on failure
//   expect := the current value), void sp_set_hdr(u32 slot, u64), void sp_put(u32 slot, const
//   Pos&), bool sp_same(u32 slot, const Pos&), u32 sp_owner_gen(u32 owner) (its generation as
//   last published; may lag, never leads), void sp_claimed() (one more slot in use),
//   void sp_fail() (no free slot within SPILL_PROBES: sticky error for the host).
// Spill entry (64 B): hdr = (owner + 1) | count << 28 | generation << 32, then 7 bitboards.
// A slot once claimed never becomes empty again (a dead entry -- its owner's generation moved
// on -- is reclaimed in place), so a probe sequence stops only at an empty slot and every live
// entry lies within SPILL_PROBES of its home.
static constexpr int SPILL_PROBES = 4096;
GC_HD u64 sp_make(u32 owner, u32 gen, u32 cnt) { return (u64)(owner + 1) | ((u64)cnt << 28) | ((u64)gen << 32); }
GC_HD u32 sp_owner1(u64 h) { return (u32)h & 0x0FFFFFFFu; }  // owner + 1 (0: empty)
GC_HD u32 sp_cnt(u64 h) { return ((u32)h >> 28) & 0xFu; }
GC_HD u32 sp_gen(u64 h) { return (u32)(h >> 32); }
GC_HD u32 sp_home(u32 key, u32 owner, u32 mask) { return ((key ^ (owner * 0x9E3779B1u)) * 0x85EBCA6Bu >> 7) & mask; }

// the count of board s in the spill part of board owner()'s window after this occurrence
// (the entry is updated), 0 if it is not there
template <class H>
GC_HD int spill_find(H& h, const Pos& s, u32 key) {
    const u32 mask = h.spill_mask(), me1 = h.owner() + 1, g = h.gen();
    u32 slot = sp_home(key, h.owner(), mask);
    for (int probe = 0; probe < SPILL_PROBES; probe++, slot = (slot + 1) & mask) {
        const u64 e = h.sp_hdr(slot);
        if (sp_owner1(e) == 0) return 0;
        if (sp_owner1(e) == me1 && sp_gen(e) == g && h.sp_same(slot, s)) {
            const u32 c = sp_cnt(e) + 1;
            h.sp_set_hdr(slot, sp_make(h.owner(), g, c));
            return (int)c;
        }
    }
    return 0;
}

// a new board of board owner()'s window into the spill table: 1, or 0 when no slot is free
// within SPILL_PROBES (sp_fail)
template <class H>
GC_HD int spill_insert(H& h, const Pos& s, u32 key) {
    const u32 mask = h.spill_mask(), g = h.gen();
    const u64 mine = sp_make(h.owner(), g, 1);
    u32 slot = sp_home(key, h.owner(), mask);
    for (int probe = 0; probe < SPILL_PROBES; probe++, slot = (slot + 1) & mask) {
        u64 e = h.sp_hdr(slot);
        for (;;) {
            const u32 o1 = sp_owner1(e);
            // free, or dead: its owner's published generation is newer than the entry's
            const bool dead = o1 != 0 && (int)(h.sp_owner_gen(o1 - 1) - sp_gen(e)) > 0;
            if (o1 != 0 && !dead) break;
            if (h.sp_cas(slot, e, mine)) {
                h.sp_put(slot, s);
                if (o1 == 0) h.sp_claimed();
                return 1;
            }  // lost the race: e is the slot's new value, look again
        }
    }
    h.sp_fail();
    return 0;
}
struct RepProbe {
    u32 key;
    RepEntry e0;  // the first probe, loaded early
};

template <class H>
GC_HD void rep_prefetch(H& h, const Pos& s, RepProbe& pr) {
    pr.key = board_key(s);
    pr.e0 = h.load((int)(pr.key & ((1u << h.bits()) - 1)));
}

// Returns how many times the board has been the pre-move board so far, this one included;
// 0 if it is new and the window is full (hist_cap).
template <class H>
GC_HD int rep_commit(H& h, const Pos& s, const RepProbe& pr, u32& hl, bool irrev) {
    const int bits = h.bits();
    const u32 size_mask = (1u << bits) - 1;
    u32 gen = h.gen();
    u32 pos = pr.key & size_mask, tag = pr.key >> bits;
    int c = 0;
    RepEntry e = pr.e0;
    for (int probe = 0; probe <= (int)size_mask; probe++) {
        if (probe) e = h.load((int)pos);
        if ((u32)e.hdr != gen) break;  // free for this generation
        if ((u32)((e.hdr >> 32) & tag_mask(bits)) == tag && rep_same(e, s)) {
            c = (int)(e.hdr >> 56) + 1;
            h.store_hdr((int)pos, (e.hdr & ~(0xFFull << 56)) | ((u64)c << 56));
            break;
        }
        pos = (pos + 1) & size_mask;
    }
    // a full table means the window spills: the rest of it is in the spill table
    const bool spilled = h.spill_mask() != 0 && (int)hl >= hist_cap(bits);
    if (!c && spilled) c = spill_find(h, s, pr.key);
    if (irrev) {  // nothing before this move can recur: clear the window
        h.bump_gen();
        hl = 0;
        return c ? c : 1;
    }
    if (c) return c;
    if (spilled) return spill_insert(h, s, pr.key);
    if ((int)hl >= hist_cap(bits)) return 0;
    RepEntry ne = {(u64)gen | ((u64)tag << 32) | (1ull << 56), s.k, s.q, s.r, s.b, s.n, s.p, s.w};
    h.store((int)pos, ne);
    hl++;
    return 1;
}

// One player_move (chess_v2.py:393-420) of the legal `action` of the side to move, with the
// engine's update_state and the next side's move list: on return 0, `s` is the new position
// (check flags, window length, M_DONE if the PRE-move board reached 3 occurrences) and
// `g`/`ms`/`scr` describe the side now to move; *mr = capture value, *rep = 3-fold verdict,
// *nchk = the side now to move is in check.  Returns 1 (state unchanged) when both kings
// end up in check (lib.rs:1442-1446), 2 (move applied, M_DONE) when the window is full.
// Never touches move_count.
// GEN: 2 = the next side's move set (gen_moves), 1 = its count only (set-wise count_moves, no
// parked targets), 0 = neither (g = gen_init of the new position; the caller counts the moves
// itself -- the single-board env lists them anyway).
template <int GEN = 2, class H, class S>
GC_HD int env_ply(Pos& s, H& hist, int action, Gen& g, MoveSet& ms, S& scr, int* mr, bool* rep, bool* nchk) {
    RepProbe pr;
    rep_prefetch(hist, s, pr);  // in flight during the move generation below
    GC_STAMP(2);
    bool white = s.meta & M_WHITE;
    Pos ns = s;
    ns.meta = (ns.meta & ~(u32)M_RIGHTS) | eff_rights(s);  // State::new
    bool irrev;
    apply_legal(ns, white, action, mr, &irrev);  // the action is legal (validated or policy-picked)
    // update_state (lib.rs:1386-1393): the side now to move's flag comes from its own
    // generation pass; the mover's flag follows from the move's legality (mover_checked).
    gen_init(ns, g);
    bool opp_chk = g.in_check;
    bool my_chk = mover_checked(s, ns, white, action);
    GC_STAMP(3);
    if (opp_chk && my_chk) return 1;
    if (GEN == 2) {
        gen_moves(ns, g, ms, scr);  // the next side's possible moves (chess_v2.py:268 / 278)
    } else {
        moveset_clear(ms);
        ms.total = GEN == 1 ? count_moves(ns, g) : 0;
    }
    GC_STAMP(4);
    u32 chk = white ? ((my_chk ? M_WCHK : 0u) | (opp_chk ? M_BCHK : 0u))
                    : ((opp_chk ? M_WCHK : 0u) | (my_chk ? M_BCHK : 0u));
    u32 hl = hl_of(s.meta);
    int c = rep_commit(hist, s, pr, hl, irrev);
    *rep = c >= 3;  // chess_v2.py:404-407
    GC_STAMP(5);
    ns.meta = with_hl((ns.meta & ~(u32)(M_WCHK | M_BCHK | M_DONE)) | chk | ((*rep || c == 0) ? M_DONE : 0u), hl);
    *nchk = opp_chk;
    s = ns;
    return c == 0 ? 2 : 0;
}

// One step() (chess_v2.py:219-294, opponent="none").  On return with o.moved, `g`/`ms`/`scr`
// describe the new position (side now to move) so the caller can pick the next action
// without regenerating.  `g0` must be gen_init(s) when VALIDATE (external actions); the
// on-device policy is trusted.
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
    int mr;
    bool rep, opp_chk;
    int rc = env_ply(s, hist, action, g, ms, scr, &mr, &rep, &opp_chk);
    if (rc == 1) {
        o.reason = R_BOTH_CHECKED;
        o.done = 1;
        return o;
    }
    o.reward = -10 + mr;  // INVALID_ACTION_REWARD + move reward (Q9)
    o.moved = 1;
    if (rep) { o.done = 1; o.reason = R_REPETITION; }
    if (rc == 2) { o.done = 1; o.reason = R_WINDOW_FULL; }
    if (ms.total == 0 && opp_chk) {  // 270-272
        s.meta |= M_DONE;
        o.done = 1;
        o.reward += 100;
        o.reason = R_MATE;
    }
    if (!o.done && !white) s.meta += (1u << M_MC_SHIFT);  // 291-292
    return o;
}

// The random opponent's pick (make_random_policy, chess_v2.py:116-127, on the device policy
// stream): rank drawn uniformly over the legal list, the k-th legal action in move-set order
// (selfplay_pick below, the same policy as the self-play driver's).
struct PolicyCtx {
    u64 seed;
    u32 board;
    u32 draw;
};

// The random self-play policy (opponent "none", reference rules): rank k drawn uniformly over
// the legal moves, the k-th in move-set order (gc_core.h sw_gen / sw_select), generated here
// set-wise from the position.  A_NONE (no draw taken) when there is no legal move.
GC_HD int selfplay_pick(const Pos& s, PolicyCtx& pc) {
    Gen g;
    gen_init(s, g);
    u64 t[SW_SETS];
    const int n = sw_gen(s, g, t);
    if (n == 0) return A_NONE;
    return sw_select(g, t, (int)policy_index(pc.seed, pc.board, pc.draw++, (u32)n));
}

// step() with the random opponent (chess_v2.py:219-294 with opponent_policy set): the
// agent's ply, WIN (+100) if the opponent is mated, else the opponent's reply (its capture
// value is subtracted), LOSS (-100) if the agent is then mated; move_count advances only
// when WHITE is to move after the step (so never for a BLACK agent, as in the reference).
// An opponent with no legal reply and no check ends the env (R_OPP_NO_MOVE; the reference's
// policy returns "resign", which maps to no action and raises).
template <bool VALIDATE, class H, class S>
GC_HD StepOut env_step_vs(Pos& s, H& hist, int action, const Gen* g0, Gen& g, MoveSet& ms, S& scr, PolicyCtx& pc) {
    StepOut o = {0, 0, R_NONE, 0};
    if (VALIDATE && !action_legal(s, *g0, action)) {
        o.reward = -10;
        o.done = (s.meta & M_DONE) ? 1 : 0;
        o.reason = R_INVALID;
        return o;
    }
    if (s.meta & M_DONE) { o.done = 1; o.reason = R_DONE_ALREADY; return o; }
    if (mc_of(s.meta) > MOVES_MAX) { o.done = 1; o.reason = R_MOVE_CAP; return o; }
    int mr;
    bool rep, chk;
    int rc = env_ply(s, hist, action, g, ms, scr, &mr, &rep, &chk);
    if (rc == 1) {
        o.reason = R_BOTH_CHECKED;
        o.done = 1;
        return o;
    }
    o.reward = -10 + mr;
    o.moved = 1;
    if (rep) { o.done = 1; o.reason = R_REPETITION; }
    if (rc == 2) { o.done = 1; o.reason = R_WINDOW_FULL; }
    if (ms.total == 0 && chk) {  // 270-272
        s.meta |= M_DONE;
        o.done = 1;
        o.reward += 100;
        o.reason = R_MATE;
    }
    if (o.done) return o;
    if (ms.total == 0) {  // 120-122: "resign" -> no action
        s.meta |= M_DONE;
        o.done = 1;
        o.reason = R_OPP_NO_MOVE;
        return o;
    }
    hist.commit();  // the agent ply's table write lands before the reply probes the table
    int oa = selfplay_pick(s, pc);  // ms.total > 0: one draw
    rc = env_ply(s, hist, oa, g, ms, scr, &mr, &rep, &chk);
    if (rc == 1) {
        o.reason = R_BOTH_CHECKED;
        o.done = 1;
        return o;
    }
    o.reward -= mr;  // 283
    if (rep) { o.done = 1; o.reason = R_REPETITION; }
    if (rc == 2) { o.done = 1; o.reason = R_WINDOW_FULL; }
    if (ms.total == 0 && chk) {  // 285-288
        s.meta |= M_DONE;
        o.done = 1;
        o.reward -= 100;
        o.reason = R_MATED;
    }
    if (s.meta & M_WHITE) s.meta += (1u << M_MC_SHIFT);  // 291-292
    return o;
}

// reset() for a BLACK agent (chess_v2.py:208-216): from the reset position (WHITE to move,
// `g`/`ms`/`scr` its move set) the opponent opens; its 3-fold verdict is discarded and
// move_count becomes 1.  With no opening move the env is left done (R_OPP_NO_MOVE).
template <class H, class S>
GC_HD void env_open_vs(Pos& s, H& hist, Gen& g, MoveSet& ms, S& scr, PolicyCtx& pc) {
    if (ms.total == 0) { s.meta |= M_DONE; return; }
    int oa = selfplay_pick(s, pc);  // one draw
    int mr;
    bool rep, chk;
    if (env_ply(s, hist, oa, g, ms, scr, &mr, &rep, &chk) == 1) { s.meta |= M_DONE; return; }
    s.meta = (s.meta & ~(u32)M_DONE) + (1u << M_MC_SHIFT);
}

}  // namespace gc
