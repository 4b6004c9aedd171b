// TEST INFRASTRUCTURE ONLY: the product's bitboard core (gym-chess_amd/csrc/gc_core.h,
// gc_env.h) compiled for the HOST with g++, so the CPU test suite can differential-test
// the exact device logic against the C oracle without a GPU.  Never shipped or loaded by
// the product (the product .so contains only device kernels + the launch shim).
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../gym-chess_amd/csrc/gc_core.h"
#include "../../gym-chess_amd/csrc/gc_env.h"

using namespace gc;

static Pos import_state(const int8_t* b, const uint8_t* m, int side_override) {
    bool white = side_override >= 0 ? side_override != 0 : m[0] != 0;
    u32 meta = (white ? M_WHITE : 0u) | (m[1] ? M_WKC : 0u) | (m[2] ? M_WQC : 0u) | (m[3] ? M_BKC : 0u) |
               (m[4] ? M_BQC : 0u) | (m[5] ? M_WCHK : 0u) | (m[6] ? M_BCHK : 0u) | ((u32)m[7] << M_MC_SHIFT);
    Pos s = from_mailbox(b, meta);
    s.meta = (s.meta & ~(u32)M_RIGHTS) | eff_rights(s);
    return s;
}
static void export_state(const Pos& s, int8_t* b, uint8_t* m) {
    to_mailbox(s, b);
    m[0] = (s.meta & M_WHITE) != 0; m[1] = (s.meta & M_WKC) != 0; m[2] = (s.meta & M_WQC) != 0;
    m[3] = (s.meta & M_BKC) != 0; m[4] = (s.meta & M_BQC) != 0; m[5] = (s.meta & M_WCHK) != 0;
    m[6] = (s.meta & M_BCHK) != 0; m[7] = (uint8_t)mc_of(s.meta);
}

extern "C" int host_list(const int8_t* b, const uint8_t* m, int white, int attack, uint16_t* out, int cap) {
    Pos s = import_state(b, m, white);
    Gen g;
    gen_init(s, g);
    int n = 0;
    u64 pcs = g.own;
    while (pcs) {
        int sq = ctz(pcs);
        pcs &= pcs - 1;
        int t = type_at(s, sq);
        u64 tg = attack ? attack_targets(s, g, sq, t) : legal_targets(s, g, sq, t);
        int c = popc(tg);
        for (int k = 0; k < c; k++) {
            if (n < cap) out[n] = (uint16_t)(sq * 64 + kth_target(tg, sq, t, g.white, k));
            n++;
        }
    }
    if (!attack) {
        if (g.castles & 1) { if (n < cap) out[n] = g.white ? A_QSW : A_QSB; n++; }
        if (g.castles & 2) { if (n < cap) out[n] = g.white ? A_KSW : A_KSB; n++; }
    }
    return n;
}

// the same list through for_targets_ordered (the device's list_one / list_par emit)
extern "C" int host_list_emit(const int8_t* b, const uint8_t* m, int white, int attack, uint16_t* out, int cap) {
    Pos s = import_state(b, m, white);
    Gen g;
    gen_init(s, g);
    int n = 0;
    for (u64 pcs = g.own; pcs; pcs &= pcs - 1) {
        int sq = ctz(pcs);
        int t = type_at(s, sq);
        u64 tg = attack ? attack_targets(s, g, sq, t) : legal_targets(s, g, sq, t);
        for_targets_ordered(tg, sq, t, g.white, [&](int to) { if (n < cap) out[n] = (uint16_t)(sq * 64 + to); n++; });
    }
    if (!attack) {
        if (g.castles & 1) { if (n < cap) out[n] = g.white ? A_QSW : A_QSB; n++; }
        if (g.castles & 2) { if (n < cap) out[n] = g.white ? A_KSW : A_KSB; n++; }
    }
    return n;
}

extern "C" int host_count(const int8_t* b, const uint8_t* m, int white) {
    Pos s = import_state(b, m, white);
    Gen g;
    gen_init(s, g);
    return count_legal(s, g);
}

extern "C" int host_select(const int8_t* b, const uint8_t* m, int white, int k) {
    Pos s = import_state(b, m, white);
    Gen g;
    gen_init(s, g);
    return select_legal(s, g, k);
}

extern "C" int host_action_legal(const int8_t* b, const uint8_t* m, int white, int a) {
    Pos s = import_state(b, m, white);
    Gen g;
    gen_init(s, g);
    return action_legal(s, g, a) ? 1 : 0;
}

extern "C" int host_next_state(const int8_t* b, const uint8_t* m, int white, int action, int8_t* ob, uint8_t* om,
                               int* reward) {
    Pos s = import_state(b, m, -1);
    bool irrev;
    int rc = apply_move(s, white != 0, action, reward, &irrev);
    if (rc == 0) {
        u32 chk = check_flags(s);
        s.meta = (s.meta & ~(u32)(M_WCHK | M_BCHK)) | chk;
        if ((chk & (M_WCHK | M_BCHK)) == (M_WCHK | M_BCHK)) rc = 1;
    }
    export_state(s, ob, om);
    return rc;
}

extern "C" void host_update_state(const int8_t* b, const uint8_t* m, int8_t* ob, uint8_t* om) {
    Pos s = import_state(b, m, -1);
    s.meta = (s.meta & ~(u32)(M_WCHK | M_BCHK)) | check_flags(s);
    export_state(s, ob, om);
}

// mover_checked (the step's shortcut for the mover's check flag) next to the full probe it
// replaces, for a legal `action` of the side to move: bit 0 = shortcut, bit 1 = full probe
extern "C" int host_mover_checked(const int8_t* b, const uint8_t* m, int action) {
    Pos s = import_state(b, m, -1);
    bool white = (s.meta & M_WHITE) != 0;
    Pos ns = s;
    int r;
    bool irrev;
    apply_legal(ns, white, action, &r, &irrev);
    int mk = tracked_king(ns, white);
    bool full = mk >= 0 && sq_attacked(ns, mk, !white);
    return (mover_checked(s, ns, white, action) ? 1 : 0) | (full ? 2 : 0);
}

// the two forms of the pin / check sets (gc_core.h gen_pins_aligned, gen_pins_part) agree
extern "C" int host_pins_agree(const int8_t* b, const uint8_t* m, int white) {
    Pos s = import_state(b, m, white);
    Gen g, h;
    gen_base(s, g);
    h = g;
    gen_pins_finish(g, gen_pins_aligned(s, g));  // the block sets differ by the checker square itself,
    gen_pins_finish(h, gen_pins_part<15, true>(s, h));  // the check masks (checkers | block) do not
    return g.in_check == h.in_check && g.checkmask == h.checkmask && g.pinned == h.pinned && g.pinrays == h.pinrays;
}
// count_moves (the perft leaves' set-wise count) == gen_moves' total == count_legal: returns
// the count, or -1 - gen_moves' total when they differ
extern "C" int host_count_moves_agree(const int8_t* b, const uint8_t* m, int white) {
    Pos s = import_state(b, m, white);
    Gen g;
    gen_init(s, g);
    MoveSet ms;
    NoScratch none;
    gen_moves(s, g, ms, none);
    int c = count_moves(s, g);
    return (c == ms.total && c == count_legal(s, g) && c == count_position(s)) ? c : -1 - ms.total;
}
// set-wise generation (the self-play policy's move-set order): the count == gen_moves' total,
// and sw_select over every rank yields each legal action exactly once.  Returns the count, or
// -1 - the first rank whose action is wrong (or -1000 - total on a count mismatch)
extern "C" int host_sw_agree(const int8_t* b, const uint8_t* m, int white) {
    Pos s = import_state(b, m, white);
    Gen g;
    gen_init(s, g);
    u64 t[SW_SETS];
    const int n = sw_gen(s, g, t);
    if (n != count_legal(s, g)) return -1000 - n;
    std::vector<char> seen(4101, 0);
    u64 cw[4] = {0, 0, 0, 0};
    sw_pack(t, 0, SW_SETS, cw);
    const int normal = n - popc(g.castles);
    for (int k = 0; k < n; k++) {
        const int a = sw_select(g, t, k);
        if (a < 0 || a > A_RESIGN || seen[a] || !action_legal(s, g, a)) return -1 - k;
        seen[a] = 1;
        if (n < 256) {  // the two-step form of the paired kernel
            int r = k, b;
            if (k < normal) {
                const int j = sw_locate(cw, r);
                b = sw_finish(g, j, t[j], r);
            } else {
                b = sw_castle(g, k - normal);
            }
            if (b != a) return -1 - k;
        }
    }
    return n;
}
// quick_legal (the paired API step's validation) == action_legal over gen_init, for every
// action id: returns the number of legal actions, or -1 - the first action that differs
extern "C" int host_quick_legal_agree(const int8_t* b, const uint8_t* m, int white) {
    Pos s = import_state(b, m, white);
    Gen g;
    gen_init(s, g);
    int n = 0;
    for (int a = -1; a <= A_RESIGN + 1; a++) {
        bool q = quick_legal(s, a), r = action_legal(s, g, a);
        bool split = quick_pseudo(s, a) && quick_safe(s, a);  // the quad API step's two halves
        if (q != r || split != r) return -1 - a;
        n += r;
    }
    for (int a : {5000, 8191, 65535})
        if (quick_legal(s, a) || (quick_pseudo(s, a) && quick_safe(s, a))) return -1 - a;
    return n;
}
extern "C" uint64_t host_between(int a, int b) { return between(a, b); }
extern "C" uint64_t host_rook_att(int sq, uint64_t occ) { return rook_att(sq, occ); }
extern "C" uint64_t host_bishop_att(int sq, uint64_t occ) { return bishop_att(sq, occ); }
extern "C" uint64_t host_side_attacks(const int8_t* b, int white) {
    uint8_t m[8] = {0};
    Pos s = import_state(b, m, 1);
    return side_attacks(s, white != 0);
}

static uint64_t perft_rec(const Pos& s, int d) {
    Gen g;
    gen_init(s, g);
    if (d <= 1) return (uint64_t)count_legal(s, g);
    uint64_t tot = 0;
    int n = count_legal(s, g);
    for (int k = 0; k < n; k++) {
        int a = select_legal(s, g, k);
        Pos c = s;
        int rw;
        bool irrev;
        apply_move(c, g.white, a, &rw, &irrev);
        c.meta = (c.meta & ~(u32)M_RIGHTS) | eff_rights(c);
        tot += perft_rec(c, d - 1);
    }
    return tot;
}
extern "C" uint64_t host_perft(const int8_t* b, const uint8_t* m, int depth) {
    Pos s = import_state(b, m, -1);
    if (depth <= 0) return 1;
    return perft_rec(s, depth);
}

// ---- env rollout on the host with the same driver as k_env_rollout ----------------------
struct HostHist {  // same contract as the device DevHist (gc_env.h rep_prefetch/rep_commit)
    std::vector<RepEntry> tabv;
    u32 g = 0;
    int nbits = HTAB_BITS;
    HostHist() : tabv(HTAB_MAX) {
        for (auto& e : tabv) e = RepEntry{0, 0, 0, 0, 0, 0, 0, 0};
    }
    int bits() const { return nbits; }
    u32 gen() const { return g; }
    void bump_gen() { g++; }
    RepEntry load(int p) const { return tabv[p]; }
    void store_hdr(int p, u64 h) { tabv[p].hdr = h; }
    void store(int p, const RepEntry& e) { tabv[p] = e; }
    void commit() {}  // host stores are immediate
    // the spill table (gc_env.h): one board, so the owner is 0 and its generation is g;
    // enabled (2^14 entries) for a BLACK agent as on the device
    std::vector<u64> spv;
    u32 spmask = 0, used = 0, failed = 0;
    void enable_spill(int bits) {
        spmask = (1u << bits) - 1;
        spv.assign((size_t)8 << bits, 0);
    }
    u32 spill_mask() const { return spmask; }
    u32 owner() const { return 0; }
    u64 sp_hdr(u32 slot) const { return spv[(size_t)slot * 8]; }
    bool sp_cas(u32 slot, u64& expect, u64 desired) {
        u64& h = spv[(size_t)slot * 8];
        if (h != expect) { expect = h; return false; }
        h = desired;
        return true;
    }
    void sp_set_hdr(u32 slot, u64 v) { spv[(size_t)slot * 8] = v; }
    void sp_put(u32 slot, const Pos& s) {
        u64* d = &spv[(size_t)slot * 8];
        d[1] = s.k; d[2] = s.q; d[3] = s.r; d[4] = s.b; d[5] = s.n; d[6] = s.p; d[7] = s.w;
    }
    bool sp_same(u32 slot, const Pos& s) const {
        const u64* d = &spv[(size_t)slot * 8];
        return d[1] == s.k && d[2] == s.q && d[3] == s.r && d[4] == s.b && d[5] == s.n && d[6] == s.p && d[7] == s.w;
    }
    u32 sp_owner_gen(u32) const { return g; }
    void sp_claimed() { used++; }
    void sp_fail() { failed = 1; }
};

struct HostScratch {
    static constexpr bool kPark = true;
    u64 v[SCRATCH_SLOTS];
    void put(int j, u64 x) { v[j] = x; }
    u64 get(int j) const { return v[j]; }
};

extern "C" int host_count2(const int8_t* b, const uint8_t* m, int white) {
    Pos s = import_state(b, m, white);
    Gen g;
    gen_init(s, g);
    MoveSet ms;
    HostScratch scr;
    gen_moves(s, g, ms, scr);
    return ms.total;
}
extern "C" int host_select2(const int8_t* b, const uint8_t* m, int white, int k) {
    Pos s = import_state(b, m, white);
    Gen g;
    gen_init(s, g);
    MoveSet ms;
    HostScratch scr;
    gen_moves(s, g, ms, scr);
    return select_move(s, g, ms, scr, k);
}
extern "C" int host_select_action(const int8_t* b, const uint8_t* m, int white, int k) {
    Pos s = import_state(b, m, white);
    Gen g;
    gen_init(s, g);
    MoveSet ms;
    HostScratch scr;
    gen_moves(s, g, ms, scr);
    return select_action(s, g, ms, scr, k);
}

static void host_reset(Pos& s, HostHist& h, const Pos& ip) {
    s = env_reset_pos(ip);
    h.bump_gen();
}

// the self-play driver of k_env_step<true, OPP> / k_env_rollout<OPP> on the host
// select_action_swar (the paired step's pick) == select_action for every rank: returns the
// number of ranks checked, or -1 - the first rank that differs
extern "C" int host_pick_agree(const int8_t* b, const uint8_t* m, int white) {
    Pos s = import_state(b, m, white);
    Gen g;
    gen_init(s, g);
    MoveSet ms;
    HostScratch scr;
    gen_moves(s, g, ms, scr);
    for (int k = 0; k < ms.total; k++)
        if (select_action_swar(s, g, ms, scr, k) != select_action(s, g, ms, scr, k)) return -1 - k;
    return ms.total;
}

struct HostEnv {
    Pos init, s;
    HostHist h;
    HostScratch scr;
    Gen g;
    MoveSet ms;
    int opp = 0, agent_black = 0;
    PolicyCtx pc = {0, 0, 0};
    void regen() {
        gen_init(s, g);
        gen_moves(s, g, ms, scr);
    }
    void reset() {
        host_reset(s, h, init);
        regen();
        if (opp && agent_black) env_open_vs(s, h, g, ms, scr, pc);
    }
    int pick() { return selfplay_pick(s, pc); }  // the random policy: move-set order
};

extern "C" void host_rollout_trace2(const int8_t* init, uint64_t seed, uint32_t board, int plies, int opp,
                                    int agent_white, int16_t* tr_action, int16_t* tr_reward, uint8_t* tr_done,
                                    uint8_t* tr_reason, int8_t* final_board, uint8_t* final_meta, uint64_t* stats8) {
    HostEnv e;
    e.init = from_mailbox(init, 0);
    e.opp = opp;
    e.agent_black = !agent_white;
    e.h.nbits = e.agent_black ? HTAB_BITS_UNCAPPED : HTAB_BITS;
    if (e.agent_black) e.h.enable_spill(14);
    e.pc = PolicyCtx{seed, board, 0};
    e.reset();
    int a = e.pick();
    uint64_t steps = 0, rsum = 0, ends[6] = {0, 0, 0, 0, 0, 0};
    for (int p = 0; p < plies; p++) {
        StepOut o = {0, 0, R_NONE, 0};
        bool have = false;
        int played = a;
        if (a == A_NONE) {
            e.reset();
            have = true;
            o.reason = R_NO_MOVES;
            ends[R_NO_MOVES]++;
            played = -1;
        } else {
            o = opp ? env_step_vs<false>(e.s, e.h, a, nullptr, e.g, e.ms, e.scr, e.pc)
                    : env_step<false>(e.s, e.h, a, nullptr, e.g, e.ms, e.scr);
            have = o.moved;
            steps++;
            rsum += (uint64_t)(int64_t)o.reward;
            if (o.done) {
                int slot = o.reason == R_MATED ? 1
                           : (o.reason == R_OPP_NO_MOVE ? 4 : (o.reason == R_WINDOW_FULL ? 5 : o.reason));
                ends[slot < 6 ? slot : 0]++;
                e.reset();
                have = true;
            }
        }
        if (!have) e.regen();
        tr_action[p] = (int16_t)played;
        tr_reward[p] = (int16_t)o.reward;
        tr_done[p] = (uint8_t)o.done;
        tr_reason[p] = (uint8_t)o.reason;
        a = e.pick();
    }
    export_state(e.s, final_board, final_meta);
    stats8[0] = steps; stats8[1] = rsum;
    for (int k = 0; k < 6; k++) stats8[2 + k] = ends[k];
}
extern "C" void host_rollout_trace(const int8_t* init, uint64_t seed, uint32_t board, int plies, int16_t* tr_action,
                                   int16_t* tr_reward, uint8_t* tr_done, uint8_t* tr_reason, int8_t* final_board,
                                   uint8_t* final_meta, uint64_t* stats8) {
    host_rollout_trace2(init, seed, board, plies, 0, 1, tr_action, tr_reward, tr_done, tr_reason, final_board,
                        final_meta, stats8);
}

// external-action env for step-by-step replay of the reference env traces
extern "C" void* host_env_new2(const int8_t* init, int opp, int agent_white, uint64_t seed, uint32_t board) {
    HostEnv* e = new HostEnv();
    e->init = from_mailbox(init, 0);
    e->opp = opp;
    e->agent_black = !agent_white;
    e->h.nbits = e->agent_black ? HTAB_BITS_UNCAPPED : HTAB_BITS;
    if (e->agent_black) e->h.enable_spill(14);
    e->pc = PolicyCtx{seed, board, 0};
    e->reset();
    return e;
}
extern "C" void* host_env_new(const int8_t* init) { return host_env_new2(init, 0, 1, 0, 0); }
extern "C" void host_env_free(void* p) { delete (HostEnv*)p; }
extern "C" void host_env_reset(void* p) { ((HostEnv*)p)->reset(); }
extern "C" int host_env_pick(void* p) {
    HostEnv* e = (HostEnv*)p;
    e->regen();
    int a = e->pick();
    return a == A_NONE ? -1 : a;
}
extern "C" uint32_t host_env_draw(void* p) { return ((HostEnv*)p)->pc.draw; }
extern "C" int host_env_step(void* p, int action, int* reward, int* done, int* reason) {
    HostEnv* e = (HostEnv*)p;
    Gen g0;
    gen_init(e->s, g0);
    StepOut o = e->opp ? env_step_vs<true>(e->s, e->h, action, &g0, e->g, e->ms, e->scr, e->pc)
                       : env_step<true>(e->s, e->h, action, &g0, e->g, e->ms, e->scr);
    *reward = o.reward;
    *done = o.done;
    *reason = o.reason;
    return o.reason == R_BOTH_CHECKED ? 1 : 0;
}
extern "C" void host_env_state(void* p, int8_t* b, uint8_t* m) { export_state(((HostEnv*)p)->s, b, m); }
extern "C" int host_env_moves(void* p, uint16_t* out, int cap) {
    HostEnv* e = (HostEnv*)p;
    int8_t b[64];
    uint8_t m[8];
    export_state(e->s, b, m);
    return host_list(b, m, -1, 0, out, cap);
}

// perft via the device algorithm (gc_perft.h): levels > 3 expanded recursively here
#include "../../gym-chess_amd/csrc/gc_perft.h"
static uint64_t perft_split(const Pos& s, int d) {
    if (d <= 3) {
        HostScratch a, b;
        return perft_small(s, d, a, b);
    }
    Gen g;
    gen_init(s, g);
    uint64_t tot = 0;
    int n = count_legal(s, g);
    for (int k = 0; k < n; k++) tot += perft_split(child_of(s, g.white, select_legal(s, g, k)), d - 1);
    return tot;
}
extern "C" uint64_t host_perft_small(const int8_t* b, const uint8_t* m, int depth) {
    Pos s = import_state(b, m, -1);
    return perft_split(s, depth);
}

// ---- FIDE rules mode (gc_fide.h), engine convention meta8[7] = en-passant file + 1 --------
#include "../../gym-chess_amd/csrc/gc_fide.h"

static Pos fide_import(const int8_t* b, const uint8_t* m) {
    u32 meta = (m[0] ? M_WHITE : 0u) | (m[1] ? M_WKC : 0u) | (m[2] ? M_WQC : 0u) | (m[3] ? M_BKC : 0u) |
               (m[4] ? M_BQC : 0u);
    meta = fide::with_ep(meta, m[7] ? (m[7] - 1) & 7 : -1);
    return from_mailbox(b, meta);
}

static uint64_t fide_perft_rec(const Pos& s, int depth) {
    if (depth <= 3) return fide::fperft_small(s, depth);
    fide::FGen f;
    fide::fgen(s, f);
    uint64_t n = 0;
    int rw;
    bool irr;
    u64 pcs = f.g.own;
    while (pcs) {
        int sq = ctz(pcs);
        pcs &= pcs - 1;
        int t = type_at(s, sq);
        u64 tg = fide::ftargets(s, f, sq, t);
        while (tg) {
            int to = ctz(tg);
            tg &= tg - 1;
            int np = (t == PAWN && (bit(to) & fide::promo_row(f.g.white))) ? 4 : 1;
            for (int pc = 0; pc < np; pc++) {
                Pos c = s;
                fide::fapply(c, sq * 64 + to, np == 4 ? QUEEN + pc : 0, &rw, &irr);
                n += fide_perft_rec(c, depth - 1);
            }
        }
    }
    for (int cb = 0; cb < 2; cb++) {
        if (!(f.g.castles & (1u << cb))) continue;
        Pos c = s;
        fide::fapply(c, cb ? (f.g.white ? A_KSW : A_KSB) : (f.g.white ? A_QSW : A_QSB), 0, &rw, &irr);
        n += fide_perft_rec(c, depth - 1);
    }
    return n;
}

// the shared generator (fcount) against the per-square walk (fcount_walk) at every node of a
// FIDE perft tree; on the first difference the node is exported to (ob, om) and 1 returned
static int fide_cmp_rec(const Pos& s, int depth, int8_t* ob, uint8_t* om, int* counts) {
    fide::FGen f;
    fide::fgen(s, f);
    int a = fide::fcount(s, f, true), w = fide::fcount_walk(s, f, true);
    {  // the set-wise generator (the FIDE self-play pick): same action count, every rank a
       // distinct legal action
        u64 t[SW_SETS];
        const int n = fide::fsw_gen(s, f, t), na = fide::fcount_walk(s, f, false);
        std::vector<char> seen(4101, 0);
        bool ok = n == na;
        for (int k = 0; ok && k < n; k++) {
            const int act = sw_select(f.g, t, k);
            ok = act >= 0 && act < 4101 && !seen[act] && fide::faction_legal(s, f, act);
            if (ok) seen[act] = 1;
        }
        if (!ok) a = -1 - n;
    }
    if (a != w) {
        to_mailbox(s, ob);
        for (int k = 0; k < 8; k++) om[k] = 0;
        om[0] = (s.meta & M_WHITE) != 0;
        counts[0] = a;
        counts[1] = w;
        counts[2] = fide::ep_square(s.meta);
        return 1;
    }
    if (depth <= 1) return 0;
    int rw;
    bool irr;
    u64 pcs = f.g.own;
    while (pcs) {
        int sq = ctz(pcs);
        pcs &= pcs - 1;
        int t = type_at(s, sq);
        u64 tg = fide::ftargets(s, f, sq, t);
        while (tg) {
            int to = ctz(tg);
            tg &= tg - 1;
            Pos c = s;
            fide::fapply(c, sq * 64 + to, (t == PAWN && (bit(to) & fide::promo_row(f.g.white))) ? QUEEN : 0, &rw, &irr);
            if (fide_cmp_rec(c, depth - 1, ob, om, counts)) return 1;
        }
    }
    for (int cb = 0; cb < 2; cb++) {
        if (!(f.g.castles & (1u << cb))) continue;
        Pos c = s;
        fide::fapply(c, cb ? (f.g.white ? A_KSW : A_KSB) : (f.g.white ? A_QSW : A_QSB), 0, &rw, &irr);
        if (fide_cmp_rec(c, depth - 1, ob, om, counts)) return 1;
    }
    return 0;
}
extern "C" int host_fide_gen_check(const int8_t* b, const uint8_t* m, int depth, int8_t* ob, uint8_t* om, int* counts) {
    return fide_cmp_rec(fide_import(b, m), depth, ob, om, counts);
}

extern "C" uint64_t host_fide_perft(const int8_t* b, const uint8_t* m, int depth) {
    return fide_perft_rec(fide_import(b, m), depth);
}

extern "C" int host_fide_list(const int8_t* b, const uint8_t* m, uint16_t* out, int cap) {
    Pos s = fide_import(b, m);
    fide::FGen f;
    fide::fgen(s, f);
    int n = 0;
    u64 pcs = f.g.own;
    while (pcs) {
        int sq = ctz(pcs);
        pcs &= pcs - 1;
        u64 tg = fide::ftargets(s, f, sq, type_at(s, sq));
        while (tg) {
            int to = ctz(tg);
            tg &= tg - 1;
            if (n < cap) out[n] = (uint16_t)(sq * 64 + to);
            n++;
        }
    }
    if (f.g.castles & 1) { if (n < cap) out[n] = f.g.white ? A_QSW : A_QSB; n++; }
    if (f.g.castles & 2) { if (n < cap) out[n] = f.g.white ? A_KSW : A_KSB; n++; }
    return n;
}

// FIDE env trajectory (random self-play driver, as k_fenv_step<true>): per-ply action,
// reward, done, reason
extern "C" void host_fide_rollout(const int8_t* init, uint64_t seed, uint32_t board, int plies, int16_t* tr_action,
                                  int16_t* tr_reward, uint8_t* tr_done, uint8_t* tr_reason) {
    Pos ip = from_mailbox(init, 0);
    auto reset = [&]() {
        Pos s = ip;
        s.meta = M_WHITE | M_RIGHTS;
        s.meta |= fide::fcheck_flags(s);
        return s;
    };
    HostHist h;
    h.bump_gen();  // zeroed entries are of generation 0: dead
    Pos s = reset();
    u32 draw = 0;
    HostScratch scr;
    auto pick = [&](const Pos& p) {
        fide::FGen f;
        fide::fgen(p, f);
        return fide::fpick_action(p, f, scr, seed, board, draw);
    };
    int a = pick(s);
    for (int p = 0; p < plies; p++) {
        StepOut o = {0, 0, R_NONE, 0};
        int played = a;
        if (a == A_NONE) {
            s = reset();
            h.bump_gen();
            o.reason = R_NO_MOVES;
            played = -1;
        } else {
            fide::FGen f;
            o = fide::fenv_step<false>(s, h, a, f);
            if (o.done) {
                s = reset();
                h.bump_gen();
            }
        }
        a = pick(s);
        tr_action[p] = (int16_t)played;
        tr_reward[p] = (int16_t)o.reward;
        tr_done[p] = (uint8_t)o.done;
        tr_reason[p] = (uint8_t)o.reason;
    }
}
