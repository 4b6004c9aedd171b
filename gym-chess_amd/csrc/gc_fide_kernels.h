// gc_fide_kernels.h -- device kernels of the optional FIDE rules mode (gc_fide.h), included
// by gymchess.hip after the shared device structures (SoA, EnvDev, DevHist).  One lane =
// one board; this mode is a correctness feature (validated by standard perft counts), so
// it uses the straightforward per-square enumeration rather than the reference mode's
// parked-target / count-plane machinery.
//
// Engine state convention in FIDE mode: meta8[7] = en-passant FILE + 1 (0 = none) instead
// of move_count (the engine calls of the reference carry no move count).
#pragma once

namespace gcf = gc::fide;

__device__ __host__ inline u32 fide_meta_from8(const uint8_t* m, bool white) {
    u32 meta = (white ? M_WHITE : 0u) | (m[1] ? M_WKC : 0u) | (m[2] ? M_WQC : 0u) | (m[3] ? M_BKC : 0u) |
               (m[4] ? M_BQC : 0u) | (m[5] ? M_WCHK : 0u) | (m[6] ? M_BCHK : 0u);
    return gcf::with_ep(meta, m[7] ? (int)(m[7] - 1) & 7 : -1);
}

__global__ void k_fimport(const int8_t* __restrict__ boards, const uint8_t* __restrict__ meta8,
                          const uint8_t* __restrict__ side, SoA out) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= out.n) return;
    const uint8_t* m = meta8 + 8 * (size_t)i;
    bool white = side ? side[i] != 0 : m[0] != 0;
    out.store(i, from_mailbox(boards + 64 * (size_t)i, fide_meta_from8(m, white)));
}

__global__ void k_fexport(SoA in, int8_t* __restrict__ boards, uint8_t* __restrict__ meta8) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= in.n) return;
    Pos s = in.load(i);
    to_mailbox(s, boards + 64 * (size_t)i);
    uint8_t* m = meta8 + 8 * (size_t)i;
    m[0] = (s.meta & M_WHITE) != 0; m[1] = (s.meta & M_WKC) != 0; m[2] = (s.meta & M_WQC) != 0;
    m[3] = (s.meta & M_BKC) != 0; m[4] = (s.meta & M_BQC) != 0; m[5] = (s.meta & M_WCHK) != 0;
    m[6] = (s.meta & M_BCHK) != 0;
    m[7] = (s.meta & gcf::M_EP) ? (uint8_t)(((s.meta & gcf::M_EP_MASK) >> gcf::M_EP_SHIFT) + 1) : 0;
}

// legal list in ascending action id, castles last (queen side, then king side, as the
// reference lists them); attack mode = the attack-mode targets of gc_core.h, no castles
__global__ void k_flist(SoA in, int attack, int cap, uint16_t* __restrict__ out, int32_t* __restrict__ counts) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= in.n) return;
    Pos s = in.load(i);
    gcf::FGen f;
    gcf::fgen(s, f);
    uint16_t* o = out + (size_t)cap * i;
    int n = 0;
    u64 pcs = f.g.own;
    while (pcs) {
        int sq = ctz(pcs);
        pcs &= pcs - 1;
        int t = type_at(s, sq);
        u64 tg = attack ? attack_targets(s, f.g, sq, t) : gcf::ftargets(s, f, sq, t);
        while (tg) {
            int to = ctz(tg);
            tg &= tg - 1;
            if (n < cap) o[n] = (uint16_t)(sq * 64 + to);
            n++;
        }
    }
    if (!attack) {
        if (f.g.castles & 1) { if (n < cap) o[n] = f.g.white ? A_QSW : A_QSB; n++; }
        if (f.g.castles & 2) { if (n < cap) o[n] = f.g.white ? A_KSW : A_KSB; n++; }
    }
    counts[i] = n;
}

__global__ void k_fmask(SoA in, u64* __restrict__ mask, int32_t* __restrict__ counts) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= in.n) return;
    Pos s = in.load(i);
    gcf::FGen f;
    gcf::fgen(s, f);
    u64* o = mask + 65 * (size_t)i;
    int n = 0;
    for (int sq = 0; sq < 64; sq++) {
        u64 tg = ((f.g.own >> sq) & 1) ? gcf::ftargets(s, f, sq, type_at(s, sq)) : 0;
        o[sq] = tg;
        n += popc(tg);
    }
    u64 c = 0;
    if (f.g.castles & 1) c |= f.g.white ? (1ull << 1) : (1ull << 3);
    if (f.g.castles & 2) c |= f.g.white ? (1ull << 0) : (1ull << 2);
    o[64] = c;
    if (counts) counts[i] = n + popc(c);
}

// next_state under FIDE rules (promotion to a queen); status 0 ok, -1 no piece of the side
// to move on the from-square, -2 bad action
__global__ void k_fnext_state(SoA in, const uint16_t* __restrict__ actions, SoA out, int32_t* __restrict__ rewards,
                              int32_t* __restrict__ status) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= in.n) return;
    Pos s = in.load(i);
    int rw = 0;
    bool irrev;
    int rc = gcf::fapply(s, actions[i], 0, &rw, &irrev);
    if (rc == 0) s.meta = (s.meta & ~(u32)(M_WCHK | M_BCHK)) | gcf::fcheck_flags(s);
    out.store(i, s);
    rewards[i] = rw;
    status[i] = rc;
}

__global__ void k_fupdate_state(SoA st) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= st.n) return;
    Pos s = st.load(i);
    s.meta = (s.meta & ~(u32)(M_WCHK | M_BCHK)) | gcf::fcheck_flags(s);
    st.store(i, s);
}

// perft levels: children counted with promotions x4, expanded in enumeration order
__global__ void k_fcount_children(SoA in, int64_t* __restrict__ cnt) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= in.n) return;
    Pos s = in.load(i);
    gcf::FGen f;
    gcf::fgen(s, f);
    cnt[i] = gcf::fcount(s, f, true);
}
// parents a .. a+c-1 of `in`, children at offs[t] (relative to the chunk's first child)
__global__ void k_fexpand_range(SoA in, int a, int c, const int64_t* __restrict__ offs, SoA out) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= c) return;
    Pos s = in.load(a + t);
    gcf::FGen f;
    gcf::fgen(s, f);
    int o = (int)offs[t];
    u64 pcs = f.g.own;
    int rw;
    bool irr;
    while (pcs) {
        int sq = ctz(pcs);
        pcs &= pcs - 1;
        int t = type_at(s, sq);
        u64 tg = gcf::ftargets(s, f, sq, t);
        while (tg) {
            int to = ctz(tg);
            tg &= tg - 1;
            int np = (t == PAWN && (bit(to) & gcf::promo_row(f.g.white))) ? 4 : 1;
            for (int pc = 0; pc < np; pc++) {
                Pos c = s;
                gcf::fapply(c, sq * 64 + to, np == 4 ? QUEEN + pc : 0, &rw, &irr);
                out.store(o++, c);
            }
        }
    }
    for (int cb = 0; cb < 2; cb++) {
        if (!(f.g.castles & (1u << cb))) continue;
        Pos c = s;
        gcf::fapply(c, cb ? (f.g.white ? A_KSW : A_KSB) : (f.g.white ? A_QSW : A_QSB), 0, &rw, &irr);
        out.store(o++, c);
    }
}
__global__ void k_fperft_small(SoA in, int depth, uint64_t* __restrict__ nodes) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= in.n) return;
    nodes[i] = gcf::fperft_small(in.load(i), depth);
}

// ---- env (opponent "none"): one lane = one board, per-square policy pick ------------------
template <class S>
__device__ uint16_t fpick(const Pos& s, const gcf::FGen& f, S& scr, uint64_t seed, int i, u32& draw) {
    return (uint16_t)gcf::fpick_action(s, f, scr, seed, (u32)i, draw);
}

__device__ Pos fide_reset_pos(const EnvDev& e) {
    Pos s = {e.init[0], e.init[1], e.init[2], e.init[3], e.init[4], e.init[5], e.init[6], 0};
    s.meta = M_WHITE | M_RIGHTS;  // chess_v2.py:194-201: all four rights at reset
    s.meta |= gcf::fcheck_flags(s);
    return s;
}

// the FIDE reset position's move set for the paired kernels (as k_init_cache for the
// reference rules): every reset lands on it
__global__ void __launch_bounds__(BLOCK) k_finit_cache(EnvDev e, EnvDev::InitCache* out, uint16_t* acts) {
    LDS_SCRATCH_DECL;
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    EnvDev::InitCache c = {};
    c.pos = fide_reset_pos(e);
    gcf::FGen f;
    gcf::fgen(c.pos, f);
    const bool walk = gcf::fuses_walk(f);
    MoveSet ms;
    moveset_clear(ms);
    if (!walk) gcf::fgen_moves(c.pos, f, ms, scr);
    c.own = f.g.own; c.fastp = ms.fastp; c.o1 = ms.o1; c.o2 = ms.o2; c.ol = ms.ol; c.orr = ms.orr;
    for (int b = 0; b < 5; b++) c.cnt[b] = ms.cnt[b];
    for (int j = 0; j < SCRATCH_SLOTS; j++) c.slots[j] = walk ? 0 : scr.get(j);
    c.total = walk ? gcf::fcount_walk(c.pos, f, false) : ms.total;
    c.castles = f.g.castles;
    c.white = f.g.white;
    c.usable = !walk;
    c.table = c.usable && c.total > 0 && c.total <= RESET_ACTS_MAX;
    if (c.table) {  // the self-play policy's move-set order (gcf::fpick_action)
        u64 t[SW_SETS];
        gcf::fsw_gen(c.pos, f, t);
        for (int k = 0; k < c.total; k++) acts[k] = (uint16_t)sw_select(f.g, t, k);
    }
    *out = c;
}

// POLICY=false: external action e.act[i] (validated); POLICY=true: the random self-play
// driver (act[i] = this state's policy pick; A_NONE or done -> reset; pick the next action).
// OPP: the random opponent replies inside the step (gcf::fenv_step_vs) and, for a BLACK agent,
// opens after every reset (gcf::fenv_open_vs), as k_env_step<POLICY, true> does.
template <bool POLICY, bool OPP = false>
__global__ void __launch_bounds__(BLOCK) k_fenv_step(EnvDev e) {
    LDS_SCRATCH_DECL;
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= e.n) return;
    Pos s = e.st.load(i);
    u32 g0 = e.hgen[i], d = e.draw[i], nst = e.nsteps[i];
    int a = (int)e.act[i];
    DevHist h = e.hist(i, g0);
    StepOut o = {0, 0, R_NONE, 0};
    gcf::FGen f;
    bool have = false;
    if (POLICY && a == A_NONE) {
        s = fide_reset_pos(e);
        h.bump_gen();
        o.reason = R_NO_MOVES;
    } else {
        o = OPP ? gcf::fenv_step_vs<!POLICY>(s, h, a, f, scr, e.seed, (u32)i, d) : gcf::fenv_step<!POLICY>(s, h, a, f);
        have = o.moved;
        nst += 1;
        if (POLICY && o.done) {
            s = fide_reset_pos(e);
            h.bump_gen();
            have = false;
        }
    }
    if (POLICY) {
        if (!have) {
            gcf::fgen(s, f);
            if (OPP && e.agent_black) gcf::fenv_open_vs(s, h, f, scr, e.seed, (u32)i, d);
        }
        e.act[i] = fpick(s, f, scr, e.seed, i, d);
    }
    e.draw[i] = d;
    h.commit();
    e.st.store(i, s);
    h.flush(g0);
    e.nsteps[i] = nst;
    e.reward[i] = o.reward;
    e.done[i] = (uint8_t)o.done;
    e.reason[i] = (uint8_t)o.reason;
}

template <bool OPP = false>
__global__ void __launch_bounds__(BLOCK) k_fenv_reset(EnvDev e, const uint8_t* __restrict__ mask, int select) {
    LDS_SCRATCH_DECL;
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= e.n) return;
    if (mask && !mask[i]) return;
    const u32 g0 = e.hgen[i];
    DevHist h = e.hist(i, g0);
    Pos s = fide_reset_pos(e);
    h.bump_gen();
    if ((OPP && e.agent_black) || select) {
        gcf::FGen f;
        gcf::fgen(s, f);
        u32 d = e.draw[i];
        if (OPP && e.agent_black) gcf::fenv_open_vs(s, h, f, scr, e.seed, (u32)i, d);
        if (select) e.act[i] = fpick(s, f, scr, e.seed, i, d);
        e.draw[i] = d;
        h.commit();
    }
    h.flush(g0);
    e.st.store(i, s);
}

// the fused random self-play under FIDE rules with the random opponent (the paired fused
// kernel serves opponent "none"): one lane per board, `plies` steps in one launch, the
// per-ply trace and stats as k_env_rollout
template <bool OPP>
__global__ void __launch_bounds__(BLOCK) k_fenv_rollout(EnvDev e, int plies, u64* trace, uint64_t* stats) {
    LDS_SCRATCH_DECL;
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= e.n) return;
    Pos s = e.st.load(i);
    u32 g0 = e.hgen[i], d = e.draw[i];
    int a = (int)e.act[i];
    DevHist h = e.hist(i, g0);
    uint64_t steps = 0, rsum = 0;
    u32 e_mate = 0, e_rep = 0, e_cap = 0, e_nomove = 0, e_err = 0;
    StepOut o = {0, 0, R_NONE, 0};
    for (int p = 0; p < plies; p++) {
        o = {0, 0, R_NONE, 0};
        gcf::FGen f;
        bool have = false;
        int played = a;
        if (a == A_NONE) {
            s = fide_reset_pos(e);
            h.bump_gen();
            o.reason = R_NO_MOVES;
            e_nomove++;
            played = -1;
        } else {
            o = OPP ? gcf::fenv_step_vs<false>(s, h, a, f, scr, e.seed, (u32)i, d) : gcf::fenv_step<false>(s, h, a, f);
            have = o.moved;
            steps++;
            rsum += (uint64_t)(int64_t)o.reward;
            if (o.done) {
                e_mate += o.reason == R_MATE || o.reason == R_MATED;
                e_rep += o.reason == R_REPETITION;
                e_cap += o.reason == R_MOVE_CAP;
                e_err += o.reason == R_WINDOW_FULL;
                e_nomove += o.reason == R_OPP_NO_MOVE;
                s = fide_reset_pos(e);
                h.bump_gen();
                have = false;
            }
        }
        if (!have) {
            gcf::fgen(s, f);
            if (OPP && e.agent_black) gcf::fenv_open_vs(s, h, f, scr, e.seed, (u32)i, d);
        }
        if (trace) trace[(size_t)p * e.n + i] = trace_word(played, o);
        a = fpick(s, f, scr, e.seed, i, d);
        h.commit();
    }
    e.reward[i] = o.reward;
    e.done[i] = (uint8_t)o.done;
    e.reason[i] = (uint8_t)o.reason;
    e.st.store(i, s);
    h.flush(g0);
    e.draw[i] = d;
    e.act[i] = (uint16_t)a;
    e.nsteps[i] += (u32)steps;
    if (stats) {
        uint64_t* so = stats + 8 * (size_t)i;
        so[0] += steps; so[1] += rsum;
        so[2 + R_MATE] += e_mate; so[2 + R_REPETITION] += e_rep; so[2 + R_MOVE_CAP] += e_cap;
        so[2 + R_NO_MOVES] += e_nomove; so[2 + R_BOTH_CHECKED] += e_err;
    }
}

__global__ void __launch_bounds__(BLOCK) k_fenv_select(EnvDev e) {
    LDS_SCRATCH_DECL;
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= e.n) return;
    Pos s = e.st.load(i);
    gcf::FGen f;
    gcf::fgen(s, f);
    u32 d = e.draw[i];
    e.act[i] = fpick(s, f, scr, e.seed, i, d);
    e.draw[i] = d;
}

// env ingest under FIDE rules: meta8 as the env's (meta8[7] = move_count), en passant from
// ep[i] (file, or -1 = none); check flags from the board
__global__ void k_fenv_import(const int8_t* __restrict__ boards, const uint8_t* __restrict__ meta8,
                              const int8_t* __restrict__ ep, EnvDev e) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= e.n) return;
    const uint8_t* m = meta8 + 8 * (size_t)i;
    u32 meta = (m[0] ? M_WHITE : 0u) | (m[1] ? M_WKC : 0u) | (m[2] ? M_WQC : 0u) | (m[3] ? M_BKC : 0u) |
               (m[4] ? M_BQC : 0u) | ((u32)m[7] << M_MC_SHIFT);
    meta = gcf::with_ep(meta, ep ? (int)ep[i] : -1);
    Pos s = from_mailbox(boards + 64 * (size_t)i, meta);
    s.meta |= gcf::fcheck_flags(s);
    e.st.store(i, s);
    e.hgen[i] += 1;
}
