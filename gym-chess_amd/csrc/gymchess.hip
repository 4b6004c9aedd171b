// gymchess.hip -- HIP kernels (gfx950) + the extern "C" boundary (include/gymchess.h).
//
// One lane = one board.  Board state lives in HBM as structure-of-arrays: bitboard j of
// board i at bb[j*N + i] (j = K,Q,R,B,N,P,W), meta[i], so every wave's loads and stores
// of one field are 512 contiguous bytes.  All move generation is register-resident
// integer/bitwise work (gc_core.h), with per-piece move targets parked in LDS for the
// ordered policy pick; the only other HBM traffic is the 3-fold repetition window
// (gc_env.h): usually one 64-byte probe of a per-board hash table, issued before move
// generation so that its latency overlaps it.
//
// The C-ABI replaces the reference's FFI (the PyO3 ChessEngine, lib.rs:1412-1512) for the
// engine calls, plus a device-resident batched env for chess_v2.py's reset()/step().
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <chrono>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#ifdef GC_STAMPS
// diagnostic build only: per-wave s_memtime stamps (MI355X guide, "In-kernel stamps")
__shared__ unsigned long long gc_stamp_lds[4][8];
__device__ __forceinline__ void gc_stamp(int k) {
    __builtin_amdgcn_sched_barrier(0);
    unsigned long long t;
#ifdef GC_STAMPS_REAL  // the 100 MHz constant clock, comparable across CUs (launch ramp / tail)
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    if (k == 0) {  // placement of the wave in bits 44+ of its first stamp: cu | sh | se | simd | xcc
        unsigned hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)\n\ts_getreg_b32 %1, hwreg(HW_REG_XCC_ID)"
                     : "=s"(hw), "=s"(xcc));
        unsigned long long where = ((hw >> 8) & 0xF) | (((hw >> 12) & 1) << 4) | (((hw >> 13) & 3) << 5) |
                                   (((hw >> 4) & 3) << 7) | ((unsigned long long)(xcc & 0xF) << 9);
        t = (t & ((1ull << 44) - 1)) | (where << 44);
    }
#else
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
#endif
    __builtin_amdgcn_sched_barrier(0);
    if ((threadIdx.x & 63) == 0) gc_stamp_lds[threadIdx.x >> 6][k] = t;
}
#define GC_STAMP(k) gc_stamp(k)
#endif
#ifdef GC_PSTAMPS
// diagnostic build only: per wave, the cycles of each segment of the fused ply (phase work
// and barrier waits), summed over the launch's plies (tools/pstamp_probe.py)
__shared__ unsigned long long gc_pst[8][9];  // [wave][segment 0..7, last stamp]
__device__ unsigned long long* g_pst_out;
__device__ __forceinline__ void gc_pst_mark(int k) {
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) {
        const int w = threadIdx.x >> 6;
        gc_pst[w][k] += t - gc_pst[w][8];
        gc_pst[w][8] = t;
    }
    __builtin_amdgcn_sched_barrier(0);
}
#define PST(k) gc_pst_mark(k)
#else
#define PST(k)
#endif
#include "gc_core.h"
#include "gc_env.h"
#include "gc_perft.h"
#include "gc_fide.h"
#include "../../include/gymchess.h"

using namespace gc;
namespace gcf = gc::fide;

#define NBB 7
#define BLOCK 256

// ----------------------------------------------------------------------------- errors
static thread_local std::string g_err;
static int fail(const std::string& m) {
    g_err = m;
    return -1;
}
#define HIPCHK(x)                                                                   \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) return fail(std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)

extern "C" const char* gc_last_error(void) { return g_err.c_str(); }
extern "C" int gc_version(void) { return GC_ABI_VERSION; }
// The build's source hash (sha256 of the sources and the compile flags, set by
// __graft_entry__.build_hip): the loader refuses a library built from other sources.
#ifndef GC_SRC_HASH
#define GC_SRC_HASH "unhashed"
#endif
extern "C" const char* gc_build_hash(void) { return "gymchess-src-hash:" GC_SRC_HASH; }
extern "C" int gc_get_device_count(int* n) {
    if (!n) return fail("null out pointer");
    HIPCHK(hipGetDeviceCount(n));
    return 0;
}

// ----------------------------------------------------------------------------- SoA access
struct SoA {
    u64* bb;   // [7][N]
    u32* meta; // [N]
    int n;
    __device__ Pos load(int i) const {
        Pos s;
        s.k = bb[0 * (size_t)n + i]; s.q = bb[1 * (size_t)n + i]; s.r = bb[2 * (size_t)n + i];
        s.b = bb[3 * (size_t)n + i]; s.n = bb[4 * (size_t)n + i]; s.p = bb[5 * (size_t)n + i];
        s.w = bb[6 * (size_t)n + i];
        s.meta = meta[i];
        return s;
    }
    __device__ void store(int i, const Pos& s) const {
        bb[0 * (size_t)n + i] = s.k; bb[1 * (size_t)n + i] = s.q; bb[2 * (size_t)n + i] = s.r;
        bb[3 * (size_t)n + i] = s.b; bb[4 * (size_t)n + i] = s.n; bb[5 * (size_t)n + i] = s.p;
        bb[6 * (size_t)n + i] = s.w;
        meta[i] = s.meta;
    }
};

// The env's spill table (gc_env.h spill_find / spill_insert): 64-B entries shared by the
// boards of a BLACK-agent env whose windows outgrow their per-board tables; ctr[0] = slots
// ever claimed, ctr[1] = sticky "no free slot" flag (both read by the host, gc_env_*).
struct SpillTab {
    u64* ent;  // [mask + 1][8]
    u32* ctr;
    u32 mask;  // 0: no spill table (every env but a BLACK agent's)
};

// repetition window of board i (gc_env.h rep_prefetch / rep_commit): HTAB 64-byte entries
// per board (entry() below), one cache line each (4 x 16-B loads); generation [N]
struct DevHist {
    u64* htab;
    u32* hgen;
    u32 g;
    int i;
    int nb = HTAB_BITS;  // log2 entries per board (gc_env.h: 9, or 10 for a BLACK agent)
    // Wave-blocked layout: entry pos of board i at ((i/64)*HTAB + pos)*64 + i%64, i.e. the 64
    // boards of a wave share one 4 MiB block and a wave's 64 probes land on 64 random 4 KiB
    // rows of it.  Board-major tables (64 KiB per board) put a wave's probes 64 KiB apart, on
    // the same HBM channels: tools/lat_probe.hip measures 9.6 vs 5.5 us per launch for one
    // random 64-B read + write per board at 65 536 boards.
    __device__ size_t entry(int pos) const { return ((((size_t)(i >> 6)) << nb) + pos) * 64 + (i & 63); }
    __device__ int bits() const { return nb; }
    __device__ u32 gen() const { return g; }
    __device__ void bump_gen() { g++; }                // written back by flush()
    __device__ void flush(u32 g0) const { if (g != g0) hgen[i] = g; }
    __device__ RepEntry load(int pos) const {
        const ulonglong2* p = reinterpret_cast<const ulonglong2*>(htab + entry(pos) * 8);
        ulonglong2 a = p[0], b = p[1], c = p[2], d = p[3];
        RepEntry e = {a.x, a.y, b.x, b.y, c.x, c.y, d.x, d.y};
        return e;
    }
    // Table writes are recorded and issued by commit() at the end of the step: a store
    // issued mid-kernel makes the compiler wait (vmcnt) before reusing its data registers.
    int wkind = 0, wpos = 0;  // 0 none, 1 header only, 2 whole entry
    RepEntry we;
    __device__ void store_hdr(int pos, u64 h) { wkind = 1; wpos = pos; we.hdr = h; }
    __device__ void store(int pos, const RepEntry& e) { wkind = 2; wpos = pos; we = e; }
    __device__ void commit() {
        u64* base = htab + entry(wpos) * 8;
        if (wkind == 1) {
            base[0] = we.hdr;
        } else if (wkind == 2) {
            ulonglong2* p = reinterpret_cast<ulonglong2*>(base);
            p[0] = make_ulonglong2(we.hdr, we.k);
            p[1] = make_ulonglong2(we.q, we.r);
            p[2] = make_ulonglong2(we.b, we.n);
            p[3] = make_ulonglong2(we.p, we.w);
        }
        wkind = 0;
    }
    // the spill table (gc_env.h): headers through device-coherent atomics -- other boards'
    // lanes, on any XCD, claim slots concurrently; a board's own entry bodies are written and
    // read only by its own lane (or by later launches)
    SpillTab sp = {nullptr, nullptr, 0};
    __device__ u32 spill_mask() const { return sp.mask; }
    __device__ u32 owner() const { return (u32)i; }
    __device__ u64 sp_hdr(u32 slot) const {
        return __hip_atomic_load(sp.ent + (size_t)slot * 8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __device__ bool sp_cas(u32 slot, u64& expect, u64 desired) const {
        return __hip_atomic_compare_exchange_strong(sp.ent + (size_t)slot * 8, &expect, desired, __ATOMIC_RELAXED,
                                                    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __device__ void sp_set_hdr(u32 slot, u64 v) const {
        __hip_atomic_store(sp.ent + (size_t)slot * 8, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __device__ void sp_put(u32 slot, const Pos& s) const {
        u64* d = sp.ent + (size_t)slot * 8;
        d[1] = s.k; d[2] = s.q; d[3] = s.r; d[4] = s.b; d[5] = s.n; d[6] = s.p; d[7] = s.w;
    }
    __device__ bool sp_same(u32 slot, const Pos& s) const {
        const u64* d = sp.ent + (size_t)slot * 8;
        return d[1] == s.k && d[2] == s.q && d[3] == s.r && d[4] == s.b && d[5] == s.n && d[6] == s.p && d[7] == s.w;
    }
    __device__ u32 sp_owner_gen(u32 o) const { return __hip_atomic_load(hgen + o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
    __device__ void sp_claimed() const { __hip_atomic_fetch_add(sp.ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
    __device__ void sp_fail() const { __hip_atomic_fetch_or(sp.ctr + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
};

// per-lane move-target scratch in LDS: slot j of lane t at lds[j*BLOCK + t] (each wave's
// ds_read_b64/ds_write_b64 touches 512 contiguous bytes: conflict-free)
struct LdsScratch {
    static constexpr bool kPark = true;
    u64* base;
    __device__ void put(int j, u64 v) { base[j * BLOCK] = v; }
    __device__ u64 get(int j) const { return base[j * BLOCK]; }
};
#define LDS_SCRATCH_DECL __shared__ u64 lds_scr[SCRATCH_SLOTS * BLOCK]; LdsScratch scr{lds_scr + threadIdx.x}

// ----------------------------------------------------------------------------- engine kernels
// import: mailbox int8[64] + meta8 {side, wkc, wqc, bkc, bqc, ...} -> bitboards, with the
// State::new rights forcing (lib.rs:295-336).  `side` may override meta8[0] (player arg).
__device__ __forceinline__ Pos import_one(const int8_t* __restrict__ boards, const uint8_t* __restrict__ meta8,
                                          const uint8_t* __restrict__ side, int i) {
    const uint8_t* m = meta8 + 8 * (size_t)i;
    bool white = side ? side[i] != 0 : m[0] != 0;
    u32 meta = (white ? M_WHITE : 0u) | (m[1] ? M_WKC : 0u) | (m[2] ? M_WQC : 0u) | (m[3] ? M_BKC : 0u) |
               (m[4] ? M_BQC : 0u) | (m[5] ? M_WCHK : 0u) | (m[6] ? M_BCHK : 0u) | ((u32)m[7] << M_MC_SHIFT);
    Pos s = from_mailbox(boards + 64 * (size_t)i, meta);
    s.meta = (s.meta & ~(u32)M_RIGHTS) | eff_rights(s);
    return s;
}
__global__ void k_import(const int8_t* __restrict__ boards, const uint8_t* __restrict__ meta8,
                         const uint8_t* __restrict__ side, SoA out) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= out.n) return;
    out.store(i, import_one(boards, meta8, side, i));
}

__device__ __forceinline__ void export_one(const Pos& s, int8_t* __restrict__ boards, uint8_t* __restrict__ meta8, int i) {
    if (boards) to_mailbox(s, boards + 64 * (size_t)i);
    if (meta8) {
        uint8_t* m = meta8 + 8 * (size_t)i;
        m[0] = (s.meta & M_WHITE) != 0; m[1] = (s.meta & M_WKC) != 0; m[2] = (s.meta & M_WQC) != 0;
        m[3] = (s.meta & M_BKC) != 0; m[4] = (s.meta & M_BQC) != 0; m[5] = (s.meta & M_WCHK) != 0;
        m[6] = (s.meta & M_BCHK) != 0; m[7] = (uint8_t)mc_of(s.meta);
    }
}
__global__ void k_export(SoA in, int8_t* __restrict__ boards, uint8_t* __restrict__ meta8) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= in.n) return;
    export_one(in.load(i), boards, meta8, i);
}

// ordered move list in reference order (lib.rs:460-563 + 1468-1479); attack mode lists the
// unfiltered attack-mode moves and no castles.  count may exceed cap (list truncated).
__device__ __forceinline__ void list_one(const Pos& s, int attack, int cap, uint16_t* __restrict__ out,
                                         int32_t* __restrict__ counts, int i) {
    Gen g;
    gen_init(s, g);
    uint16_t* o = out + (size_t)cap * i;
    int n = 0;
    u64 pcs = g.own;
    while (pcs) {
        int sq = ctz(pcs);
        pcs &= pcs - 1;
        int t = type_at(s, sq);
        u64 tg = attack ? attack_targets(s, g, sq, t) : legal_targets(s, g, sq, t);
        for_targets_ordered(tg, sq, t, g.white, [&](int to) { if (n < cap) o[n] = (uint16_t)(sq * 64 + to); n++; });
    }
    if (!attack) {
        if (g.castles & 1) { if (n < cap) o[n] = g.white ? A_QSW : A_QSB; n++; }
        if (g.castles & 2) { if (n < cap) o[n] = g.white ? A_KSW : A_KSB; n++; }
    }
    counts[i] = n;
}
// list_one with the wave's 64 lanes (every lane holds the same s): lane = square, each own
// piece's legal targets in reference order at its exclusive prefix-sum offset (the list is
// row-major over the squares, lib.rs:501-563), the castles after them
// (attack: the attack-mode list, lib.rs:460-486 with attack = true -- no legality filter, no
// castles)
__device__ __forceinline__ void list_par(const Pos& s, int cap, uint16_t* out, int32_t* count, const Gen* g0 = nullptr,
                                         bool attack = false) {
    Gen g;
    if (g0) g = *g0;  // (gen_init of s, made by the caller)
    else gen_init(s, g);
    const int sq = (int)(threadIdx.x & 63);
    const bool mine = (g.own >> sq) & 1;
    const int t = mine ? type_at(s, sq) : 0;
    const u64 tg = mine ? (attack ? attack_targets(s, g, sq, t) : legal_targets(s, g, sq, t)) : 0ull;
    const int c = popc(tg);
    int off = c;  // inclusive prefix sum over the lanes
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int v = __shfl_up(off, d, 64);
        if (sq >= d) off += v;
    }
    const int n = __shfl(off, 63, 64);
    off -= c;
    int w = off;
    for_targets_ordered(tg, sq, t, g.white, [&](int to) { if (w < cap) out[w] = (uint16_t)(sq * 64 + to); w++; });
    int m = n;
    if (sq == 0) {
        if (!attack && (g.castles & 1)) { if (m < cap) out[m] = g.white ? A_QSW : A_QSB; m++; }
        if (!attack && (g.castles & 2)) { if (m < cap) out[m] = g.white ? A_KSW : A_KSB; m++; }
        *count = m;
    }
}

__global__ void k_list(SoA in, int attack, int cap, uint16_t* __restrict__ out, int32_t* __restrict__ counts) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= in.n) return;
    list_one(in.load(i), attack, cap, out, counts, i);
}
// the engine calls' one-launch forms (reference rules): mailbox in, the op, mailbox out -- a
// single-board call pays one launch instead of three
__global__ void k_list_mb(const int8_t* __restrict__ boards, const uint8_t* __restrict__ meta8,
                          const uint8_t* __restrict__ side, int n, int attack, int cap, uint16_t* __restrict__ out,
                          int32_t* __restrict__ counts) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    list_one(import_one(boards, meta8, side, i), attack, cap, out, counts, i);
}

// legal action mask: 64 words (from-square -> target bitboard) + 1 word of castle bits
// (bit c set <=> action 4096+c legal)
__global__ void k_mask(SoA in, u64* __restrict__ mask, int32_t* __restrict__ counts) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= in.n) return;
    Pos s = in.load(i);
    Gen g;
    gen_init(s, g);
    u64* o = mask + 65 * (size_t)i;
    int n = 0;
    for (int sq = 0; sq < 64; sq++) {
        u64 tg = ((g.own >> sq) & 1) ? legal_targets(s, g, sq, type_at(s, sq)) : 0;
        o[sq] = tg;
        n += popc(tg);
    }
    u64 c = 0;
    if (g.castles & 1) c |= g.white ? (1ull << 1) : (1ull << 3);
    if (g.castles & 2) c |= g.white ? (1ull << 0) : (1ull << 2);
    o[64] = c;
    if (counts) counts[i] = n + popc(c);
}

// the castle bits alone (k_mask's word 64): what get_castle_moves returns
__global__ void k_castle_word(SoA in, int32_t* __restrict__ out) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= in.n) return;
    Pos s = in.load(i);
    Gen g;
    gen_init(s, g);
    int c = 0;
    if (g.castles & 1) c |= g.white ? (1 << 1) : (1 << 3);
    if (g.castles & 2) c |= g.white ? (1 << 0) : (1 << 2);
    out[i] = c;
}

// next_state (lib.rs:1422-1452): move + update_state; status 0 ok, 1 both kings checked,
// -1 empty from-square (reference panics), -2 bad action
__device__ __forceinline__ Pos next_state_one(Pos s, const uint8_t* __restrict__ player_white,
                                              const uint16_t* __restrict__ actions, int32_t* __restrict__ rewards,
                                              int32_t* __restrict__ status, int i) {
    int rw = 0;
    bool irrev;
    int rc = apply_move(s, player_white[i] != 0, actions[i], &rw, &irrev);
    if (rc == 0) {
        u32 chk = check_flags(s);
        s.meta = (s.meta & ~(u32)(M_WCHK | M_BCHK)) | chk;
        if ((chk & (M_WCHK | M_BCHK)) == (M_WCHK | M_BCHK)) rc = 1;
    }
    rewards[i] = rw;
    status[i] = rc;
    return s;
}
__global__ void k_next_state(SoA in, const uint8_t* __restrict__ player_white, const uint16_t* __restrict__ actions,
                             SoA out, int32_t* __restrict__ rewards, int32_t* __restrict__ status) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= in.n) return;
    out.store(i, next_state_one(in.load(i), player_white, actions, rewards, status, i));
}
// mailbox in and out (in place: a thread reads and writes only its own board)
__global__ void k_next_state_mb(int8_t* __restrict__ boards, uint8_t* __restrict__ meta8,
                                const uint8_t* __restrict__ player_white, const uint16_t* __restrict__ actions, int n,
                                int32_t* __restrict__ rewards, int32_t* __restrict__ status) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    export_one(next_state_one(import_one(boards, meta8, nullptr, i), player_white, actions, rewards, status, i),
               boards, meta8, i);
}

// update_state (lib.rs:1502-1511)
__global__ void k_update_state(SoA st) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= st.n) return;
    Pos s = st.load(i);
    s.meta = (s.meta & ~(u32)(M_WCHK | M_BCHK)) | check_flags(s);
    st.store(i, s);
}

// ----------------------------------------------------------------------------- perft
// Leaves: one lane = one subtree of depth <= 3 (gc_perft.h).  Interior levels: expand every
// node of a level into its children (count, exclusive scan, write), level by level, until
// the subtrees are small enough and numerous enough to fill the chip; then sum back up.
#define PERFT_MAXD 8

__global__ void __launch_bounds__(BLOCK) k_perft_small(SoA in, int depth, uint64_t* __restrict__ nodes) {
    __shared__ u64 lds_a[SCRATCH_SLOTS * BLOCK];
    __shared__ u64 lds_b[SCRATCH_SLOTS * BLOCK];
    LdsScratch sa{lds_a + threadIdx.x};
    LdsScratch sb{lds_b + threadIdx.x};
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= in.n) return;
    nodes[i] = perft_small(in.load(i), depth, sa, sb);
}

// The same over a permutation of the subtrees: perft_small's outer loop runs the subtree
// root's move count, so lanes of one wave given roots of equal count (perm = roots sorted by
// it) do not idle through the wave's longest list.  (PMC: 56 % lane utilisation unsorted.)
__global__ void __launch_bounds__(BLOCK) k_perft_small_perm(SoA in, const int32_t* __restrict__ perm, int depth,
                                                            uint64_t* __restrict__ nodes) {
    __shared__ u64 lds_a[SCRATCH_SLOTS * BLOCK];
    __shared__ u64 lds_b[SCRATCH_SLOTS * BLOCK];
    LdsScratch sa{lds_a + threadIdx.x};
    LdsScratch sb{lds_b + threadIdx.x};
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= in.n) return;
    int j = perm[i];
    nodes[j] = perft_small(in.load(j), depth, sa, sb);
}
#ifndef PERFT2_WPE
#define PERFT2_WPE 3  // 168 VGPRs: 3 waves per SIMD -- 1.12e12 nodes/s vs 1.06 at 4 (128 VGPRs, ~110 spilled) and 1.03 at 2
#endif
// The split leaf pass (perft_split_leaves) keeps its depth-2 subtree roots as one 64-byte
// record each (7 bitboards + meta: one cache line) instead of 7 + 1 SoA rows: the leaf
// kernel visits them in the order of a sort by move count, so every root is a gather --
// one line per root here, eight with the SoA rows (PMC r02: 370 B per subtree).
struct alignas(64) Node64 {
    u64 k, q, r, b, n, p, w;
    u32 meta, parent;  // parent: the root's parent in the chunk (its count is added there)
};
__device__ __forceinline__ Pos node_load(const Node64* __restrict__ v, size_t j) {
    const ulonglong2* x = reinterpret_cast<const ulonglong2*>(v + j);
    const ulonglong2 a = x[0], b = x[1], c = x[2], d = x[3];
    return Pos{a.x, a.y, b.x, b.y, c.x, c.y, d.x, (u32)d.y};
}
__device__ __forceinline__ void node_store(Node64* __restrict__ v, size_t j, const Pos& s, u32 parent) {
    ulonglong2* x = reinterpret_cast<ulonglong2*>(v + j);
    x[0] = make_ulonglong2(s.k, s.q);
    x[1] = make_ulonglong2(s.r, s.b);
    x[2] = make_ulonglong2(s.n, s.p);
    x[3] = make_ulonglong2(s.w, (u64)s.meta | ((u64)parent << 32));
}
__global__ void k_iota(int32_t* __restrict__ v, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = i;
}

// children of every node, written at offs[i] .. offs[i]+cnt[i] (offs = exclusive scan).
// T = int32_t for radix-sort keys, int64_t for level sizes (a level's child total can pass
// 2^31: depth 6 over 65 536 mid-game roots has ~3e9 nodes at its fourth level).
template <class T>
__global__ void k_count_children(SoA in, T* __restrict__ cnt) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= in.n) return;
    Pos s = in.load(i);
    Gen g;
    gen_init(s, g);
    cnt[i] = (T)count_moves(s, g);
}
// expand the parents a .. a+c-1 of `in` into `out` at offs[t] (offs indexed from a, relative
// to the chunk's first child; a chunk holds < 2^31 children)
template <class T>
__global__ void k_expand_range(SoA in, int a, int c, const T* __restrict__ offs, SoA out) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= c) return;
    Pos s = in.load(a + t);
    Gen g;
    gen_init(s, g);
    int o = (int)offs[t];
    u64 pcs = g.own;
    while (pcs) {
        int sq = ctz(pcs);
        pcs &= pcs - 1;
        u64 tg = legal_targets(s, g, sq, type_at(s, sq));
        while (tg) {
            int tt = ctz(tg);
            tg &= tg - 1;
            out.store(o++, child_of(s, g.white, sq * 64 + tt));
        }
    }
    if (g.castles & 1) out.store(o++, child_of(s, g.white, g.white ? A_QSW : A_QSB));
    if (g.castles & 2) out.store(o++, child_of(s, g.white, g.white ? A_KSW : A_KSB));
}
// the same into 64-byte records (the split leaf pass)
__global__ void k_expand_range_rec(SoA in, int a, int c, const int32_t* __restrict__ offs, Node64* __restrict__ out) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= c) return;
    Pos s = in.load(a + t);
    Gen g;
    gen_init(s, g);
    size_t o = (size_t)offs[t];
    u64 pcs = g.own;
    while (pcs) {
        int sq = ctz(pcs);
        pcs &= pcs - 1;
        u64 tg = legal_targets(s, g, sq, type_at(s, sq));
        while (tg) {
            int tt = ctz(tg);
            tg &= tg - 1;
            node_store(out, o++, child_of(s, g.white, sq * 64 + tt), (u32)t);
        }
    }
    if (g.castles & 1) node_store(out, o++, child_of(s, g.white, g.white ? A_QSW : A_QSB), (u32)t);
    if (g.castles & 2) node_store(out, o++, child_of(s, g.white, g.white ? A_KSW : A_KSB), (u32)t);
}

// The split pass's depth-2 roots placed in move-count order as they are made (round 3), so
// the leaf kernel reads them in order -- one coalesced 64-B record per lane, no gather through
// a sorted permutation (PMC r03_v5: 137 B per subtree, the 64-B records fetched as random
// 128-B lines).  A counting sort over the expansion: pass A (k_expand_count) generates every
// chunk parent's children, counts each child's moves and keeps per-block histograms
// [bin][block]; an exclusive scan of those gives every (bin, block) its range; pass B
// (k_expand_place) generates the children again and writes each record at its bin's next slot
// of its block's range (an LDS cursor per bin: the order within a bin and block is arbitrary,
// which no sum depends on).  Counts past the last bin share it (never in play: > 254 moves).
#define SPLIT_BINS 256
template <class F>
__device__ __forceinline__ void for_each_child(const Pos& s, const Gen& g, F&& f) {
    u64 pcs = g.own;
    while (pcs) {
        int sq = ctz(pcs);
        pcs &= pcs - 1;
        u64 tg = legal_targets(s, g, sq, type_at(s, sq));
        while (tg) {
            int tt = ctz(tg);
            tg &= tg - 1;
            f(child_of(s, g.white, sq * 64 + tt));
        }
    }
    if (g.castles & 1) f(child_of(s, g.white, g.white ? A_QSW : A_QSB));
    if (g.castles & 2) f(child_of(s, g.white, g.white ? A_KSW : A_KSB));
}
// the child's move count (perft2's fused count, the side to move's king lines from the parent)
__device__ __forceinline__ int split_bin(const Pos& ch, const KingLines& kl) {
    const int n = count_position_kl(ch, kl);
    return n < SPLIT_BINS - 1 ? n : SPLIT_BINS - 1;
}
__global__ void __launch_bounds__(BLOCK) k_expand_count(SoA in, int a, int c, uint8_t* __restrict__ bins,
                                                        const int32_t* __restrict__ offs, u32* __restrict__ hist,
                                                        int nblk) {
    __shared__ u32 h[SPLIT_BINS];
    for (int b = threadIdx.x; b < SPLIT_BINS; b += blockDim.x) h[b] = 0;
    __syncthreads();
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < c) {
        const Pos s = in.load(a + t);
        Gen g;
        gen_init(s, g);
        size_t o = (size_t)offs[t];
        const KingLines kl = king_lines_of(s, !g.white);  // every child's side to move, its king unmoved
        for_each_child(s, g, [&](const Pos& ch) {
            const int b = split_bin(ch, kl);
            bins[o++] = (uint8_t)b;
            atomicAdd(&h[b], 1u);
        });
    }
    __syncthreads();
    for (int b = threadIdx.x; b < SPLIT_BINS; b += blockDim.x) hist[(size_t)b * nblk + blockIdx.x] = h[b];
}
__global__ void __launch_bounds__(BLOCK) k_expand_place(SoA in, int a, int c, const uint8_t* __restrict__ bins,
                                                        const int32_t* __restrict__ offs,
                                                        const u32* __restrict__ base, int nblk,
                                                        Node64* __restrict__ out) {
    __shared__ u32 cur[SPLIT_BINS];
    for (int b = threadIdx.x; b < SPLIT_BINS; b += blockDim.x) cur[b] = base[(size_t)b * nblk + blockIdx.x];
    __syncthreads();
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= c) return;
    const Pos s = in.load(a + t);
    Gen g;
    gen_init(s, g);
    size_t o = (size_t)offs[t];
    for_each_child(s, g, [&](const Pos& ch) {
        const u32 slot = atomicAdd(&cur[bins[o++]], 1u);
        node_store(out, slot, ch, (u32)t);
    });
}
// one lane = one depth-2 subtree, the records in move-count order (k_expand_place)
__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(PERFT2_WPE)))
k_perft2_rec(const Node64* __restrict__ in, int n, unsigned long long* __restrict__ parent_sum) {
    __shared__ u64 lds_a[SCRATCH_SLOTS * BLOCK];
    LdsScratch sa{lds_a + threadIdx.x};
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const u32 parent = reinterpret_cast<const u32*>(in + i)[15];
    atomicAdd(parent_sum + parent, (unsigned long long)perft2(node_load(in, i), sa));
}

// Transpositions among the depth-2 roots (round 4): a chunk's ply-3 records repeat -- m1, x,
// m3 and m3, x, m1 reach one position -- ~1.7 records per distinct position over mid-game
// roots.  perft2 is a function of the Pos alone, so one record per position (its leader) is
// counted and the others (followers) add the leader's count into their own parents.  With
// the merge the chunk's records are written in expansion order (k_expand_range_rec) and grouped
// by sorting (below).  (Round 4's first form -- one CAS per record into an open-addressed table,
// ~1 TB/s of random line traffic, 12.5 ms per chunk -- and round 5's sort with a follower pass of
// its own were measured slower and removed in round 6.)
__device__ __forceinline__ u64 pos_hash(const Pos& s) {
    u64 h = s.meta * 0x9E3779B97F4A7C15ull;
    const u64 f[7] = {s.k, s.q, s.r, s.b, s.n, s.p, s.w};
#pragma unroll
    for (int k = 0; k < 7; k++) {
        h ^= f[k] + 0x632BE59BD9B4E019ull + (h << 6) + (h >> 2);
        h *= 0xBF58476D1CE4E5B9ull;
    }
    return h ^ (h >> 31);
}
__device__ __forceinline__ bool pos_equal(const Pos& a, const Pos& b) {
    return ((a.k ^ b.k) | (a.q ^ b.q) | (a.r ^ b.r) | (a.b ^ b.b) | (a.n ^ b.n) | (a.p ^ b.p) | (a.w ^ b.w)) == 0 &&
           a.meta == b.meta;
}
// The transposition pass by sorting (round 5): every record's 32-bit hash tag and index sorted
// by the tag (hipCUB radix sort: ~2 ms for 2^26 pairs), so equal positions are adjacent and the
// pass reads sequentially.
//   k_dedup_keys     per record, in order: the tag, the index, the leaf's move-count bin
//   (sort)           by the tag (stable: a run's members in record order)
//   k_dedup_runs_f   one lane per sorted record: the members compared whole with the run's
//                    first (and, after a tag collision, with the run's earlier members), so a
//                    merge is exact; each group's first member leads
//   k_leader_hist_f  per-block leader histograms by bin (k_place_leaders_f's blocks)
//   k_place_leaders_f  the leaders copied into move-count order
//   k_perft2_val     the leaf over the placed leaders, each lane crediting its followers
#define DEDUP_BLOCK 1024
#define DEDUP_R 1  // records per thread of the histogram / placement passes (2 or 4: no gain, round 5)
__global__ void __launch_bounds__(BLOCK) k_dedup_keys(const Node64* __restrict__ in, int n, u32* __restrict__ keys,
                                                      u32* __restrict__ vals, uint8_t* __restrict__ bins) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const Pos s = node_load(in, i);
    keys[i] = (u32)(pos_hash(s) >> 32);
    vals[i] = (u32)i;
    bins[i] = (uint8_t)split_bin(s, king_lines_of(s, (s.meta & M_WHITE) != 0));
}
// The followers credited by their leader's lane in the leaf: no follower pass, no kept counts.  k_dedup_runs_f writes, per record, a lead word (bit 31: it leads;
// bits 27-30: how many later members its run holds, GC_RUN_CAP = that many or more; bits 0-26: its sorted
// position) and, in sorted order, each member's (leader position, parent) pair; the leaf lane of
// the leader at sorted position pL walks the later members of its run -- none for a lone position,
// which then reads nothing more -- and adds its count into the parent of every member it leads.
#ifndef RUN_LEN_SHIFT
#define RUN_LEN_SHIFT 27  // sorted positions below 2^27 (chunks of up to 2^21 parents), run lengths in bits 27-30
#endif
#ifndef GC_RUN_CAP
#define GC_RUN_CAP ((1 << (31 - RUN_LEN_SHIFT)) - 1)  // the lead word's run length saturates here (a test
                                                      // build lowers it: the tag walk then runs)
#endif
static_assert(GC_RUN_CAP >= 1 && GC_RUN_CAP < (1 << (31 - RUN_LEN_SHIFT)), "GC_RUN_CAP: the bits above RUN_LEN_SHIFT");
__global__ void __launch_bounds__(BLOCK) k_dedup_runs_f(const Node64* __restrict__ in, int n,
                                                        const u32* __restrict__ keys, const u32* __restrict__ vals,
                                                        u32* __restrict__ leadw, uint2* __restrict__ fw) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const u32 k = keys[p];
    const u32 r = vals[p];
    int p0 = p;
    while (p0 > 0 && keys[p0 - 1] == k) p0--;
    u32 lp = (u32)p, parent = 0;
    if (p0 < p) {  // a later member: the earliest equal member leads
        const Pos s = node_load(in, r);
        parent = reinterpret_cast<const u32*>(in + r)[15];
        if (pos_equal(s, node_load(in, vals[p0]))) {
            lp = (u32)p0;
        } else {
            for (int t = p0 + 1; t < p; t++)
                if (pos_equal(node_load(in, vals[t]), s)) { lp = (u32)t; break; }
        }
    }
    if (lp == (u32)p) {  // a leader: the later members of its run (the walk's length in the leaf);
        // a follower's word stays as zeroed before the pass (no scattered write for it)
        int q = p + 1;
        while (q < n && q - p <= GC_RUN_CAP && keys[q] == k) q++;
        leadw[r] = 0x80000000u | ((u32)(q - p - 1) << RUN_LEN_SHIFT) | (u32)p;
    }
    fw[p] = make_uint2(lp, parent);
}
__global__ void __launch_bounds__(DEDUP_BLOCK) k_leader_hist_f(int n, const u32* __restrict__ leadw,
                                                               const uint8_t* __restrict__ bins, u32* __restrict__ hist,
                                                               int nblk) {
    __shared__ u32 hb[SPLIT_BINS];
    for (int b = threadIdx.x; b < SPLIT_BINS; b += blockDim.x) hb[b] = 0;
    __syncthreads();
    for (int r = 0; r < DEDUP_R; r++) {  // k_place_leaders_f's blocks: DEDUP_BLOCK * DEDUP_R records
        const size_t i = (size_t)blockIdx.x * DEDUP_BLOCK * DEDUP_R + (size_t)r * DEDUP_BLOCK + threadIdx.x;
        if (i < (size_t)n && (leadw[i] >> 31)) atomicAdd(&hb[bins[i]], 1u);
    }
    __syncthreads();
    for (int b = threadIdx.x; b < SPLIT_BINS; b += blockDim.x) hist[(size_t)b * nblk + blockIdx.x] = hb[b];
}
__global__ void __launch_bounds__(DEDUP_BLOCK) k_place_leaders_f(const Node64* __restrict__ in, int n,
                                                                 const uint8_t* __restrict__ bins,
                                                                 const u32* __restrict__ leadw,
                                                                 const u32* __restrict__ base, int nblk,
                                                                 Node64* __restrict__ out, u32* __restrict__ spos) {
    __shared__ u32 cur[SPLIT_BINS];
    for (int b = threadIdx.x; b < SPLIT_BINS; b += blockDim.x) cur[b] = base[(size_t)b * nblk + blockIdx.x];
    __syncthreads();
    for (int r = 0; r < DEDUP_R; r++) {
        const size_t i = (size_t)blockIdx.x * DEDUP_BLOCK * DEDUP_R + (size_t)r * DEDUP_BLOCK + threadIdx.x;
        if (i >= (size_t)n) continue;
        const u32 w = leadw[i];
        if (!(w >> 31)) continue;
        const u32 slot = atomicAdd(&cur[bins[i]], 1u);
        const ulonglong2* x = reinterpret_cast<const ulonglong2*>(in + i);
        ulonglong2* y = reinterpret_cast<ulonglong2*>(out + slot);
        const ulonglong2 r0 = x[0], r1 = x[1], r2 = x[2], r3 = x[3];
        y[0] = r0; y[1] = r1; y[2] = r2; y[3] = r3;
        spos[slot] = w & 0x7FFFFFFFu;
    }
}

// one lane = one placed leader (move-count order); its count added into its own parent and into
// the parents of the followers it leads
__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(PERFT2_WPE)))
k_perft2_val(const Node64* __restrict__ in, int n, unsigned long long* __restrict__ parent_sum, int nrec,
             const u32* __restrict__ keys, const uint2* __restrict__ fw, const u32* __restrict__ spos) {
    __shared__ u64 lds_a[SCRATCH_SLOTS * BLOCK];
    LdsScratch sa{lds_a + threadIdx.x};
    // the knight jumps from an LDS table (a read per own knight instead of the eight jump sets):
    // 1.871 -> 1.901e12 same-box (VERDICT r04 missing #3); the enemy king's neighbourhood from a
    // table lost (1.852e12)
    __shared__ u64 ntab_s[64];
    if (threadIdx.x >= 64 && threadIdx.x < 128) ntab_s[threadIdx.x - 64] = knight_set(bit((int)threadIdx.x - 64));
    __syncthreads();
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const u32 parent = reinterpret_cast<const u32*>(in + i)[15];
    const uint64_t c = perft2(node_load(in, i), sa, ntab_s);
    atomicAdd(parent_sum + parent, (unsigned long long)c);
    const u32 w = spos[i];
    const u32 pl = w & ((1u << RUN_LEN_SHIFT) - 1u);
    const int rl = (int)(w >> RUN_LEN_SHIFT);  // later members of the run (GC_RUN_CAP: that many or more)
    for (int j = (int)pl + 1; j <= (int)pl + rl; j++) {  // (nothing read for a lone position)
        const uint2 f = fw[j];
        if (f.x == pl) atomicAdd(parent_sum + f.y, (unsigned long long)c);
    }
    if (rl == GC_RUN_CAP) {  // a longer run: the rest by its tag
        const u32 k = keys[pl];
        for (int j = (int)pl + GC_RUN_CAP + 1; j < nrec && keys[j] == k; j++) {
            const uint2 f = fw[j];
            if (f.x == pl) atomicAdd(parent_sum + f.y, (unsigned long long)c);
        }
    }
}
// parent value = sum of its children's values (children of one parent are contiguous)
template <class T>
__global__ void k_sum_children(const T* __restrict__ offs, const T* __restrict__ cnt,
                               const uint64_t* __restrict__ child, int n, uint64_t* __restrict__ out) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t s = 0;
    const T c = cnt[i], o = offs[i];
    for (T k = 0; k < c; k++) s += child[o + k];
    out[i] = s;
}

// ----------------------------------------------------------------------------- env kernels
struct OpenCache;  // (k_init_open_cache)
struct EnvDev {
    SoA st;
    u64* htab;       // [N/64][HTAB][64][8] repetition tables (gc_env.h; DevHist::entry)
    u32* hgen;
    u32* draw;       // policy draws per board (Philox counter)
    uint16_t* act;   // next action per board (A_NONE = no legal move)
    int32_t* reward;
    uint8_t* done;
    uint8_t* reason;
    u32* nsteps;     // env.step() calls, per board
    u64 init[NBB];   // 7 bitboards of the initial board (kernel argument: scalar loads)
    uint64_t seed;
    int n;
    int opp;          // 0: opponent "none"; 1: the random opponent replies inside step()
    int agent_black;  // player_color BLACK (needs opp): the opponent opens at every reset
    const uint16_t* reset_acts;  // the start position's legal actions in action-id order
                                 // (RESET_ACTS_MAX; valid when ic.table): a reset board's pick
                                 // is one table read
    // Every reset lands on the same position: its state, move set and parked targets are
    // computed once at env creation (k_init_cache) and passed here by value.
    struct InitCache {
        Pos pos;
        u64 own, fastp, o1, o2, ol, orr;
        u64 cnt[5];
        u64 slots[SCRATCH_SLOTS];
        int total;
        u32 castles;
        int white;
        int usable;  // 0: the start position needs the per-square fallback (> 16 pieces)
        int table;   // reset_acts holds all `total` actions
        int open_safe;  // no opening move leaves both kings in check (paired BLACK-agent kernel)
        // not the start position's: the env's spill table, carried in this device-memory
        // block because the paired kernels' arguments are full (rewritten when it grows)
        SpillTab spill;
        // a BLACK agent's resets: the position after each opening of the move-set-order table
        // (k_init_open_cache; null until a BLACK agent is set), the agent's picks per opening
        const OpenCache* open;
        const uint16_t* open_acts;  // [opening][RESET_ACTS_MAX], action-id order
        // the fused rollout's completion word (gc_env_wait_rollout): workgroups finished
        // (device), launches finished (device), the last count written to host-mapped memory
        struct DoneWord {
            u32* ctr;
            u32* seq;
            u32* host;
        } done;
    } ic;
    int hbits;        // log2 window-table entries per board (DevHist::nb)
    __device__ DevHist hist(int i, u32 g) const {
        DevHist h{htab, hgen, g, i, hbits};
        h.sp = ic.spill;
        return h;
    }
};

// The env's per-board fields live in ONE allocation (the "slab"), at offsets that are a
// function of n only, so a kernel needs a single base pointer for all of them:
//   [0, 56n) bitboards K Q R B N P W (SoA) | meta u32 | hgen u32 | draw u32 | nsteps u32 |
//   reward i32 | act u16 | done u8 | reason u8            = 80 B per board
struct Slab {
    static constexpr size_t BYTES_PER_BOARD = 80;
    __host__ __device__ static size_t meta(size_t n) { return 56 * n; }
    __host__ __device__ static size_t hgen(size_t n) { return 60 * n; }
    __host__ __device__ static size_t draw(size_t n) { return 64 * n; }
    __host__ __device__ static size_t nsteps(size_t n) { return 68 * n; }
    __host__ __device__ static size_t reward(size_t n) { return 72 * n; }
    __host__ __device__ static size_t act(size_t n) { return 76 * n; }
    __host__ __device__ static size_t done(size_t n) { return 78 * n; }
    __host__ __device__ static size_t reason(size_t n) { return 79 * n; }
};

// Keep a loaded value in a VGPR from here on.  The per-board inputs are all loaded at kernel
// entry and pinned, so they cost ONE round trip; otherwise the compiler sinks each load to
// its first use, and because vmcnt retires in order, the wait for such a late load also
// drains the repetition-table probe that is meant to stay in flight during move generation.
__device__ __forceinline__ void pin(u64& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void pin(u32& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void pin(Pos& s) {
    pin(s.k); pin(s.q); pin(s.r); pin(s.b); pin(s.n); pin(s.p); pin(s.w); pin(s.meta);
}

__device__ Pos init_pos(const u64* init) {
    Pos s = {init[0], init[1], init[2], init[3], init[4], init[5], init[6], 0};
    return env_reset_pos(s);
}

// reset (chess_v2.py:183-206); the generation bump empties the repetition window
__device__ void reset_board(const EnvDev& e, Pos& s, DevHist& h) {
    s = e.ic.pos;
    h.bump_gen();
}

// move set of the current position: cached for a freshly reset board, else generated
__device__ void moves_after_reset(const EnvDev& e, const Pos& s, Gen& g, MoveSet& ms, LdsScratch& scr) {
    if (!e.ic.usable) {
        gen_init(s, g);
        gen_moves(s, g, ms, scr);
        return;
    }
    g.white = e.ic.white;
    g.own = e.ic.own;
    g.castles = e.ic.castles;
    ms.fastp = e.ic.fastp; ms.o1 = e.ic.o1; ms.o2 = e.ic.o2; ms.ol = e.ic.ol; ms.orr = e.ic.orr;
#pragma unroll
    for (int b = 0; b < 5; b++) ms.cnt[b] = e.ic.cnt[b];
    ms.total = e.ic.total;
    ms.big = false;
#pragma unroll
    for (int j = 0; j < SCRATCH_SLOTS; j++) scr.put(j, e.ic.slots[j]);
}

#define RESET_ACTS_MAX 128
__global__ void __launch_bounds__(BLOCK) k_init_cache(EnvDev e, EnvDev::InitCache* out, uint16_t* acts) {
    LDS_SCRATCH_DECL;
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    EnvDev::InitCache c = {};
    c.pos = init_pos(e.init);
    Gen g;
    MoveSet ms;
    gen_init(c.pos, g);
    gen_moves(c.pos, g, ms, scr);
    c.own = g.own; c.fastp = ms.fastp; c.o1 = ms.o1; c.o2 = ms.o2; c.ol = ms.ol; c.orr = ms.orr;
    for (int b = 0; b < 5; b++) c.cnt[b] = ms.cnt[b];
    for (int j = 0; j < SCRATCH_SLOTS; j++) c.slots[j] = ms.big ? 0 : scr.get(j);
    // fast pawns' targets in their slots too (select_action / write_mask read them from the
    // origin sets; the paired API step's square-major mask reads every own piece's slot)
    for (u64 fp = ms.big ? 0 : ms.fastp; fp; fp &= fp - 1) {
        const int sq = ctz(fp);
        c.slots[ordinal(g.own, sq)] = fast_pawn_targets(ms, sq, g.white);
    }
    c.total = ms.total;
    c.castles = g.castles;
    c.white = g.white;
    c.usable = !ms.big;
    c.table = c.usable && ms.total > 0 && ms.total <= RESET_ACTS_MAX;
    c.open_safe = 1;
    if (c.table) {  // the self-play policy's order (move sets), RESET_ACTS_MAX further on
        u64 t[SW_SETS];
        sw_gen(c.pos, g, t);
        for (int k = 0; k < ms.total; k++) acts[RESET_ACTS_MAX + k] = (uint16_t)sw_select(g, t, k);
    }
    for (int k = 0; c.table && k < ms.total; k++) {
        const int a = select_action(c.pos, g, ms, scr, k);
        acts[k] = (uint16_t)a;
        // env_ply's both-checked end (lib.rs:1442-1446) after this opening: the one-wave
        // kernels handle it (env_open_vs), the paired one does not
        Pos ns = c.pos;
        ns.meta = (ns.meta & ~(u32)M_RIGHTS) | eff_rights(c.pos);
        int mr;
        bool irrev;
        apply_legal(ns, c.white != 0, a, &mr, &irrev);
        Gen g2;
        gen_init(ns, g2);
        if (g2.in_check && mover_checked(c.pos, ns, c.white != 0, a)) c.open_safe = 0;
    }
    *out = c;
}

// The position after the k-th opening of the reset position's move-set-order table (the
// opponent's WHITE opening of a BLACK agent's reset, chess_v2.py:208-216), settled as the env
// settles it -- check flags, the window after it (the reset position's entry unless the opening
// is irreversible: length 1 or 0), the move count -- and the agent's moves there, as InitCache.
struct OpenCache {
    Pos pos;
    u64 own;
    u64 slots[SCRATCH_SLOTS];
    int total;
    u32 castles;
    int white;
    int usable;  // 0: > 16 own pieces (the per-piece fallback)
    int table;   // open_acts holds all `total` actions
    int irrev;   // the opening is irreversible (the window restarts empty)
};
__global__ void __launch_bounds__(BLOCK) k_init_open_cache(EnvDev e, const EnvDev::InitCache* ic,
                                                           const uint16_t* sw_tab, OpenCache* out,
                                                           uint16_t* acts) {
    LDS_SCRATCH_DECL;
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= ic->total || !ic->table) return;
    const Pos s0 = ic->pos;
    const int op = (int)sw_tab[k];
    Pos p = s0;
    p.meta = (p.meta & ~(u32)M_RIGHTS) | eff_rights(s0);  // State::new
    int mr = 0;
    bool irrev = false;
    apply_legal(p, true, op, &mr, &irrev);
    const bool mchk = mover_checked(s0, p, true, op);
    Gen g;
    MoveSet ms;
    gen_init(p, g);
    const u32 chk = (mchk ? M_WCHK : 0u) | (g.in_check ? M_BCHK : 0u);
    const u32 hl = irrev ? 0u : hl_of(s0.meta) + 1u;  // rep_commit on a fresh window: count 1
    OpenCache c = {};
    c.pos = p;
    c.pos.meta = with_hl((p.meta & ~(u32)(M_WCHK | M_BCHK | M_DONE)) | chk, hl) + (1u << M_MC_SHIFT);
    gen_moves(p, g, ms, scr);
    c.own = g.own;
    for (int j = 0; j < SCRATCH_SLOTS; j++) c.slots[j] = ms.big ? 0 : scr.get(j);
    for (u64 fp = ms.big ? 0 : ms.fastp; fp; fp &= fp - 1) {
        const int sq = ctz(fp);
        c.slots[ordinal(g.own, sq)] = fast_pawn_targets(ms, sq, g.white);
    }
    c.total = ms.total;
    c.castles = g.castles;
    c.white = g.white;
    c.usable = !ms.big;
    c.table = c.usable && ms.total > 0 && ms.total <= RESET_ACTS_MAX;
    c.irrev = irrev ? 1 : 0;
    for (int j = 0; c.table && j < ms.total; j++)
        acts[(size_t)k * RESET_ACTS_MAX + j] = (uint16_t)select_action(p, g, ms, scr, j);
    out[k] = c;
}

// the API step's `pick` output: uniform over the legal actions, the k-th in action-id order
// (the order of its legal-action mask; gc_core.h select_action)
__device__ uint16_t pick_mask_order(const Pos& s, const Gen& g, const MoveSet& ms, const LdsScratch& scr,
                                    uint64_t seed, int i, u32& draw) {
    if (ms.total == 0) return (uint16_t)A_NONE;
    u32 k = policy_index(seed, (u32)i, draw++, (u32)ms.total);
    return (uint16_t)select_action(s, g, ms, scr, (int)k);
}
// the random policy (self-play and the opponent modes): uniform, the k-th legal action in
// move-set order (gc_env.h selfplay_pick: regenerated set-wise from the position)
__device__ uint16_t pick(const Pos& s, uint64_t seed, int i, u32& draw) {
    PolicyCtx pc = {seed, (u32)i, draw};
    const int a = selfplay_pick(s, pc);
    draw = pc.draw;
    return (uint16_t)a;
}

// after a reset: the move set of the side to move; a BLACK agent's opponent opens first
template <bool OPP>
__device__ void after_reset(const EnvDev& e, Pos& s, DevHist& h, Gen& g, MoveSet& ms, LdsScratch& scr,
                            PolicyCtx& pc) {
    moves_after_reset(e, s, g, ms, scr);
    if (OPP && e.agent_black) env_open_vs(s, h, g, ms, scr, pc);
}

template <bool OPP>
__global__ void __launch_bounds__(BLOCK) k_env_reset(EnvDev e, const uint8_t* __restrict__ mask, int select) {
    LDS_SCRATCH_DECL;
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= e.n) return;
    if (mask && !mask[i]) return;
    u32 g0 = e.hgen[i];
    DevHist h = e.hist(i, g0);
    Pos s;
    reset_board(e, s, h);
    PolicyCtx pc = {e.seed, (u32)i, e.draw[i]};
    if ((OPP && e.agent_black) || select) {
        Gen g;
        MoveSet ms;
        if (OPP) {
            after_reset<OPP>(e, s, h, g, ms, scr, pc);
            if (select) e.act[i] = pick(s, e.seed, i, pc.draw);
        } else {
            e.act[i] = (uint16_t)selfplay_pick(s, pc);
        }
        h.commit();
        e.draw[i] = pc.draw;
    }
    h.flush(g0);
    e.st.store(i, s);
}

// set_states ingest for the env: import + empty window
// checks != 0: the check flags come from update_state (lib.rs:1386-1393) instead of meta8
__global__ void k_env_import(const int8_t* __restrict__ boards, const uint8_t* __restrict__ meta8, EnvDev e,
                             int checks) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= e.n) return;
    const uint8_t* m = meta8 + 8 * (size_t)i;
    u32 meta = (m[0] ? M_WHITE : 0u) | (m[1] ? M_WKC : 0u) | (m[2] ? M_WQC : 0u) | (m[3] ? M_BKC : 0u) |
               (m[4] ? M_BQC : 0u) | (m[5] ? M_WCHK : 0u) | (m[6] ? M_BCHK : 0u) | ((u32)m[7] << M_MC_SHIFT);
    Pos s = from_mailbox(boards + 64 * (size_t)i, meta);
    if (checks) s.meta = (s.meta & ~(u32)(M_WCHK | M_BCHK)) | check_flags(s);
    e.st.store(i, s);
    e.hgen[i] += 1;  // empty the repetition window
}

// One env ply per board.
//  POLICY=false: external action e.act[i], validated like chess_v2.py:240; no auto-reset.
//  POLICY=true : the random-self-play driver of test_benchmark.py -- act[i] was picked by
//                the policy from this state; A_NONE (empty move list) -> driver reset
//                without a step; done -> reset; then pick the next action.
#ifdef GC_STAMPS
__device__ unsigned long long* g_stamp_out;
#endif
template <bool POLICY, bool OPP>
__global__ void __launch_bounds__(BLOCK) k_env_step(EnvDev e) {
    LDS_SCRATCH_DECL;
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= e.n) return;
    GC_STAMP(0);
    Pos s = e.st.load(i);
    u32 g0 = e.hgen[i], d = (POLICY || OPP) ? e.draw[i] : 0u, nst = e.nsteps[i], ua = e.act[i];
    pin(s); pin(g0); pin(d); pin(nst); pin(ua);
    GC_STAMP(1);
    DevHist h = e.hist(i, g0);
    PolicyCtx pc = {e.seed, (u32)i, d};
    int a = (int)ua;
    StepOut o = {0, 0, R_NONE, 0};
    Gen g;
    MoveSet ms;
    bool have = false;
    if (POLICY && a == A_NONE) {
        reset_board(e, s, h);
        o.reason = R_NO_MOVES;
    } else {
        if (POLICY) {
            o = OPP ? env_step_vs<false>(s, h, a, nullptr, g, ms, scr, pc) : env_step<false>(s, h, a, nullptr, g, ms, scr);
        } else {
            Gen g0;
            gen_init(s, g0);
            o = OPP ? env_step_vs<true>(s, h, a, &g0, g, ms, scr, pc) : env_step<true>(s, h, a, &g0, g, ms, scr);
        }
        have = o.moved;
        nst += 1;
        if (POLICY && o.done) {
            reset_board(e, s, h);
            have = false;
        }
    }
    if (POLICY) {
        if (OPP) {
            if (!have) after_reset<OPP>(e, s, h, g, ms, scr, pc);
            GC_STAMP(6);
            e.act[i] = pick(s, e.seed, i, pc.draw);
        } else {
            e.act[i] = (uint16_t)selfplay_pick(s, pc);
        }
    }
    if (POLICY || OPP) e.draw[i] = pc.draw;
    h.commit();
    GC_STAMP(7);
#ifdef GC_STAMPS
    if (POLICY && g_stamp_out != nullptr && (threadIdx.x & 63) == 0)
        for (int k = 0; k < 8; k++) g_stamp_out[(size_t)(i >> 6) * 8 + k] = gc_stamp_lds[threadIdx.x >> 6][k];
#endif
    e.st.store(i, s);
    h.flush(g0);
    e.nsteps[i] = nst;
    e.reward[i] = o.reward;
    e.done[i] = (uint8_t)o.done;
    e.reason[i] = (uint8_t)o.reason;
}

// ----------------------------------------------------------------------------- paired step
// k_env_step2: the bench path (policy-driven self-play, opponent "none") with TWO waves per
// 64 boards.  A lone wave issues a VALU instruction at most every 4 cycles while a SIMD-32
// takes 2 per wave64 instruction (MI355X_MICROARCH.md, 'vector-instruction ISSUE cost'), so
// one wave per SIMD -- 65 536 boards on 256 CUs -- leaves half the issue slots empty and
// every memory/LDS wait exposed.  Here lane l of wave 0 and lane l of wave 1 share board l
// and split its ply into two independent instruction streams (wave-uniform roles, no
// divergence), exchanging through LDS at barriers:
//
//   phase 0   W0: applies the action (post-move board to LDS)
//             W1: issues the 3-fold window probe of the pre-move board, the Philox word of the
//                 next draw, the read of a reset board's pick from the start-position table
//                 (a serial multiply chain, hidden behind W0's move)
//   ---- barrier
//   phase 1   W0: checkers, check mask, pins (from the aligned enemy sliders), the enemy's
//                 diagonal slider attacks
//             W1: the enemy's leaper and orthogonal slider attacks, the mover's own check flag
//   ---- barrier: W0 gets the rest of the enemy map and the mover-check, W1 the check mask /
//                 pins
//   phase 2   W0: castles, pawns, knights, kings, queens (gen_moves_a)
//             W1: bishops, rooks (gen_moves_b), then the 3-fold commit (the probe has landed)
//   ---- barrier: partial count planes / totals / 3-fold count exchanged
//   phase 3   both: the step's outcome (reward, done, reason, move count, reset) --
//             identical arithmetic on identical data; W0: the policy pick (k-th legal
//             action in action-id order); W1: state, window and output stores.
//
// Results are bit-identical to k_env_step<true, false> (same gc_core/gc_env functions,
// same order of decisions; tests/test_gpu_parity.py compares both with the oracle).
#define PAIR_BOARDS 64
#ifndef PAIRS_WG
#ifndef GC_PAIR_FAIR
#define GC_PAIR_FAIR 1  // 0: A/B (k_env_rollout2's workgroups taking turns)
#endif
#define PAIRS_WG 2  // board pairs (64 boards, two waves) per workgroup: 1 -> 9.8 us per ply, 2 -> 9.3, 4 -> 10.6
#endif
struct PairLds {
    union {
        struct {
            u64 slots[SCRATCH_SLOTS][PAIR_BOARDS];  // parked targets (both waves write, W0 reads)
            u64 planes[2][5][PAIR_BOARDS];          // partial bit-sliced counts per wave
        };
        u64 sets[SW_SETS][PAIR_BOARDS];  // SW: the next side's move sets (both waves write, W0 reads one)
    };
    u64 swc[2][PAIR_BOARDS];                // SW, W1 -> W0: its sets' byte counts (words 1 and 2)
    u64 pin3[3][PAIR_BOARDS];               // W0 -> W1: checkmask, pinned, pinrays
    u64 enemy[PAIR_BOARDS];                 // W1 -> W0: enemy leaper + orthogonal attacks
    u32 f0[PAIR_BOARDS];                    // W0 -> W1: in_check
    u32 f1[PAIR_BOARDS];                    // W1 -> W0: my_chk
    u32 part[2][PAIR_BOARDS];               // partial move totals per wave
    u32 rep[PAIR_BOARDS];                   // W1 -> W0: 3-fold count c | window length << 8
    u32 act[PAIR_BOARDS];                   // W0 -> W1: the next action (fused rollout)
    u32 draw[PAIR_BOARDS];                  // W0 -> W1: the next draw counter (fused rollout)
    u64 ns[NBB][PAIR_BOARDS];               // W0 -> W1: the post-move board (phase 0)
    u32 nmeta[PAIR_BOARDS];
    int32_t mr[PAIR_BOARDS];                //           its capture reward
    u32 irrev[PAIR_BOARDS];                 //           irreversible move (3-fold window reset)
    u32 x0[PAIR_BOARDS];                    // W1 -> W0: the Philox word of the next draw
    u32 ra[PAIR_BOARDS];                    // W1 -> W0: the start-position table pick
    u64 ep[PAIR_BOARDS];                    // W1 -> W0: own pawns with a legal en-passant capture (FIDE)
};
struct PairScratch {
    static constexpr bool kPark = true;
    u64* base;
    __device__ void put(int j, u64 v) { base[j * PAIR_BOARDS] = v; }
    __device__ u64 get(int j) const { return base[j * PAIR_BOARDS]; }
};
// LDS writes of this wave complete, then the workgroup barrier.  Deliberately NOT
// __syncthreads(): its fence would also drain vmcnt, i.e. wait for W1's window probe that
// is meant to stay in flight through phase 1.
__device__ __forceinline__ void pair_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

#ifdef GC_WPE  // diagnostic builds: register budget of the paired kernels
#define PAIR_ATTR __attribute__((amdgpu_waves_per_eu(GC_WPE)))
#else
#define PAIR_ATTR
#endif
// Per-launch constants of the paired kernels (SGPRs).
struct PairCtx {
    uint64_t seed;
    u64* htab;
    u32* hgen;
    const uint16_t* racts;  // the start position's actions (reset picks), valid when rtable
    const EnvDev::InitCache* icd;  // the start position's move set (device memory)
    bool rtable;
    u32 rtotal;
};

// One half-ply of the paired driver for board i (lane l of this role's wave): the move `a`
// of the side to move in s (applied when mv) and everything env_ply (gc_env.h) derives from
// it -- the post-move board, the next side's generation (count planes of both waves merged,
// W0's parked targets in LDS), check flags, the 3-fold commit of the pre-move board (W1; its
// table write left deferred in h).  Phases 0-2 and the exchange that opens phase 3:
// w1_issue() runs on W1 in phase 0 behind the probe, w1_late() on W1 at the end of phase 2.
// With ACT_LDS, W1 reads the action from act_lds[l] after phase 0 (W0 picked it: the
// opponent's reply); with MV_LDS, whether it is played from mv_lds[l] (W0 validated it: the
// API step).  regen: a board whose move is not played gets the moves of s itself.
// FIDE = rules "fide" (gc_fide.h): fapply, the enemy map without the own king, en passant,
// FIDE castling (from W0, which alone holds the in-check flag), no king captures; a legal
// move never leaves the mover in check, so there is no mover-check and no both-checked end.
struct PairHalf {
    Pos ns;         // the post-move board (check flags / window length / done not yet set)
    Gen g;          // the next side's generation (W0 complete; W1: in_check, check mask, pins)
    MoveSet ms;     // merged count planes and total (castles included)
    int mr;         // capture reward of the move
    bool irrev;     // irreversible move (3-fold window reset)
    bool my_chk;    // the mover is in check after its move (lib.rs:1386-1393)
    bool opp_chk;   // the side now to move is in check
    bool both;      // both checked (lib.rs:1442-1446): the move is void
    bool mv;        // the move was played (MV_LDS: as W0 decided)
    int c;          // 3-fold count of the pre-move board (0: window full)
    u32 hl;         // window length after the commit
    u64 ep_from;    // FIDE: own pawns with a legal en-passant capture
    int ep;
    u64 T[SW_SETS];  // SW: the next side's move sets (each wave its own; all in LDS after phase 2)
    u64 cw[4];       // SW, W0: every set's count, one byte per set (gc_core.h sw_pack)
};
struct PairNoop {
    __device__ void operator()() const {}
};
// A role known at compile time (the fused kernels run one loop per role): every `role` test
// in the pair driver folds, so a wave's loop holds only its own role's code -- no role
// branches, and nothing the other role alone needs (the stats on W0, the pick on W1).
template <int R>
struct RoleC {
    static constexpr int value = R;
    __device__ constexpr operator int() const { return R; }
};

template <bool FIDE, bool ACT_LDS, bool MV_LDS = false, bool SW = false, class RT = int, class W1Issue, class W1Late>
__device__ __forceinline__ void pair_half(PairLds& L, RT role, int l, bool mv, bool regen, const Pos& s, int a,
                                          const u32* act_lds, const u32* mv_lds, DevHist& h, PairHalf& H,
                                          W1Issue&& w1_issue, W1Late&& w1_late) {
    PairScratch scr{&L.slots[0][l]};
    const bool white = (s.meta & M_WHITE) != 0;
    int mr = 0;
    bool irrev = false;
    Pos ns;
    RepProbe pr;
    bool my_chk = false;

    // ---- phase 0: W0 applies the action (once per board, not once per wave); W1 issues the
    // window probe of the pre-move board (Q8) and the caller's independent work
    if (role == 0) {
        ns = s;
        if constexpr (FIDE) {
            if (mv) gcf::fapply(ns, a, 0, &mr, &irrev);
        } else {
            ns.meta = (ns.meta & ~(u32)M_RIGHTS) | eff_rights(s);  // State::new
            if (mv) apply_legal(ns, white, a, &mr, &irrev);
        }
        L.ns[0][l] = ns.k; L.ns[1][l] = ns.q; L.ns[2][l] = ns.r; L.ns[3][l] = ns.b;
        L.ns[4][l] = ns.n; L.ns[5][l] = ns.p; L.ns[6][l] = ns.w;
        L.nmeta[l] = ns.meta;
        L.mr[l] = mr;
        L.irrev[l] = irrev ? 1u : 0u;
    } else {
        if (mv) rep_prefetch(h, s, pr);
        w1_issue();
    }
    PST(0);
    pair_barrier();
    PST(1);

    // ---- phase 1: W0 pins / checkers and the enemy's diagonal slider attacks; W1 the enemy's
    // leaper and orthogonal slider attacks and the mover's own check flag (FIDE: en passant)
    Gen& g = H.g;
    u64 ep_from = 0;
    int ep = -1;
    u64 enemy_diag = 0;
    if (role == 0) {
        gen_base(ns, g);
        if constexpr (FIDE) {  // FIDE positions hold one king per side: the first one (gcf::fgen)
            u64 myk = ns.k & g.own;
            g.ks = myk ? ctz(myk) : -1;
        }
        gen_pins(ns, g);
        L.pin3[0][l] = g.checkmask;
        L.pin3[1][l] = g.pinned;
        L.pin3[2][l] = g.pinrays;
        L.f0[l] = g.in_check ? 1u : 0u;
        if (g.ks >= 0) {
            if constexpr (FIDE) {  // without the own king: no retreat along a checking ray
                Pos t = ns;
                t.k &= ~(ns.k & g.own);
                t.w &= ~(ns.k & g.own);
                enemy_diag = side_attacks_diag(t, !g.white);
            } else {
                enemy_diag = side_attacks_diag(ns, !g.white);
            }
        }
    } else {
        if constexpr (ACT_LDS) a = (int)act_lds[l];
        if constexpr (MV_LDS) mv = mv_lds[l] != 0;
        ns.k = L.ns[0][l]; ns.q = L.ns[1][l]; ns.r = L.ns[2][l]; ns.b = L.ns[3][l];
        ns.n = L.ns[4][l]; ns.p = L.ns[5][l]; ns.w = L.ns[6][l];
        ns.meta = L.nmeta[l];
        mr = L.mr[l];
        irrev = L.irrev[l] != 0;
        gen_base(ns, g);
        if constexpr (FIDE) {
            u64 myk = ns.k & g.own;
            g.ks = myk ? ctz(myk) : -1;
            if (g.ks >= 0) {  // enemy map with the own king removed: no retreat along a checking ray
                Pos t = ns;
                t.k &= ~myk;
                t.w &= ~myk;
                g.enemy_att = side_attacks_leapers(t, !g.white) | side_attacks_orth(t, !g.white);
            }
            int ept = gcf::ep_square(ns.meta);  // en passant: legal captures (gcf::fgen)
            if (ept >= 0) {
                int capsq = g.white ? ept + 8 : ept - 8;
                u64 cand = pawn_att_set(bit(ept), !g.white) & ns.p & g.own;
                bool ok = (ns.p & g.opp & bit(capsq)) && !(g.occ & bit(ept));
                while (ok && cand) {
                    int fr = ctz(cand);
                    cand &= cand - 1;
                    u64 occ2 = (g.occ ^ bit(fr) ^ bit(capsq)) | bit(ept);
                    if (g.ks < 0 || !gcf::king_hit(ns, g.ks, g.white, occ2, g.opp & ~bit(capsq))) ep_from |= bit(fr);
                }
            }
            L.enemy[l] = g.enemy_att;
            L.ep[l] = ep_from;
        } else {
            if (g.ks >= 0) g.enemy_att = side_attacks_leapers(ns, !g.white) | side_attacks_orth(ns, !g.white);
            my_chk = mv && mover_checked(s, ns, white, a);
            L.enemy[l] = g.enemy_att;
            L.f1[l] = my_chk ? 1u : 0u;
        }
    }
    GC_STAMP(2);
    PST(2);
    pair_barrier();
    PST(3);
    GC_STAMP(3);

    // ---- phase 2
    if (role == 0) {
        g.enemy_att = L.enemy[l] | enemy_diag;
        if constexpr (FIDE) {
            ep_from = L.ep[l];
            if (g.ks >= 0) {  // FIDE castling: rights, king and rook home, path empty and unattacked
                const u64 myk = ns.k & g.own;
                const int base = g.white ? 56 : 0;
                bool kok = (myk & bit(base + 4)) && !g.in_check;
                u64 myr = ns.r & g.own, A = g.enemy_att, occ = g.occ;
                bool ksr = (ns.meta & (g.white ? M_WKC : M_BKC)) != 0, qsr = (ns.meta & (g.white ? M_WQC : M_BQC)) != 0;
                bool kside = kok && ksr && (myr & bit(base + 7)) && !(occ & (3ull << (base + 5))) && !(A & (3ull << (base + 5)));
                bool qside = kok && qsr && (myr & bit(base)) && !(occ & (7ull << (base + 1))) && !(A & (3ull << (base + 2)));
                g.castles = (qside ? 1u : 0u) | (kside ? 2u : 0u);
            }
        } else {
            gen_castles(ns, g);  // lib.rs:578-610 with the whole enemy map
            my_chk = L.f1[l] != 0;
        }
    } else {
        g.checkmask = L.pin3[0][l];
        g.pinned = L.pin3[1][l];
        g.pinrays = L.pin3[2][l];
        g.in_check = L.f0[l] != 0;
    }
    if constexpr (FIDE) {
        ep = ep_from ? gcf::ep_square(ns.meta) : -1;
    }
    const bool opp_chk = g.in_check;
    const bool both = !FIDE && opp_chk && my_chk;             // lib.rs:1442-1446
    const bool gen = (mv && !both) || (regen && !mv);
    MoveSet& ms = H.ms;
    moveset_clear(ms);
    ms.big = popc(g.own) > SCRATCH_SLOTS;
    int part = 0;
    int c = 0;
    u32 hl = hl_of(s.meta);
    if (role == 0) {
        if constexpr (SW) {  // pawn, knight and king sets; castles counted here (diagonal sets moved
                             // here from W1 measured within noise in round 3)
            constexpr int W0_FROM = SW_K;  // W0's sets: [0, SW_ORTH) and [SW_K, SW_SETS)
            H.cw[0] = H.cw[1] = H.cw[2] = H.cw[3] = 0;
            if (gen) {
                if constexpr (FIDE) {
                    gcf::fsw_gen_a(ns, gcf::FGen{g, ep_from, ep}, H.T);
                } else {
                    sw_pawns(ns, g, H.T);
                    sw_knights(ns, g, H.T);
                    sw_kings(ns, g, H.T);
                }
                sw_pack(H.T, 0, SW_ORTH, H.cw);
                sw_pack(H.T, W0_FROM, SW_SETS, H.cw);
                part = sw_popc(H.T, 0, SW_ORTH) + sw_popc(H.T, W0_FROM, SW_SETS) + popc(g.castles);
#pragma unroll
                for (int j = 0; j < SW_ORTH; j++) L.sets[j][l] = H.T[j];
#pragma unroll
                for (int j = W0_FROM; j < SW_SETS; j++) L.sets[j][l] = H.T[j];
            }
        } else if constexpr (FIDE) {  // castles counted here (W1 does not know them)
            if (gen) {
                if (ms.big) {
                    gcf::FGen f{g, ep_from, ep};
                    part = gcf::fcount_walk(ns, f, false);
                } else {
                    part = gen_moves_a<PairScratch, true>(ns, g, ms, scr, FideExtra{ep_from, ep}) + popc(g.castles);
                }
            }
        } else {  // castles counted here (W1 does not know them)
            if (gen) part = ms.big ? count_legal(ns, g) : gen_moves_a(ns, g, ms, scr) + popc(g.castles);
        }
    } else {
        if constexpr (SW) {  // the slider direction sets and their byte counts, to W0 through LDS
            constexpr int W1_TO = SW_K;  // W1's sets: [SW_ORTH, SW_K)
            u64 cw[4] = {0, 0, 0, 0};
            if (gen) {
                if constexpr (FIDE) {
                    gcf::fsw_gen_b(ns, gcf::FGen{g, 0, -1}, H.T);
                } else {
                    sw_orth(ns, g, H.T);
                    sw_diag_part<0, 4>(ns, g, H.T);
                }
                sw_pack(H.T, SW_ORTH, W1_TO, cw);
                part = sw_popc(H.T, SW_ORTH, W1_TO);
#pragma unroll
                for (int j = SW_ORTH; j < W1_TO; j++) L.sets[j][l] = H.T[j];
            }
            L.swc[0][l] = cw[1];
            L.swc[1][l] = cw[2];
        } else if (gen && !ms.big) {
            part = FIDE ? gen_moves_b<PairScratch, true>(ns, g, ms, scr) : gen_moves_b(ns, g, ms, scr);
        }
        if (mv && !both) {
            // the probe's data is first touched here (an opaque use after the generation:
            // otherwise the compiler hoists the entry compare up to the load and waits there)
            pin(pr.e0.hdr); pin(pr.e0.k); pin(pr.e0.q); pin(pr.e0.r);
            pin(pr.e0.b); pin(pr.e0.n); pin(pr.e0.p); pin(pr.e0.w);
            c = rep_commit(h, s, pr, hl, irrev);  // table write deferred to h.commit()
        }
        L.rep[l] = (u32)c | (hl << 8);
        w1_late();
    }
    if constexpr (!SW) {
#pragma unroll
        for (int b = 0; b < 5; b++) L.planes[role][b][l] = ms.cnt[b];
    }
    L.part[role][l] = (u32)part;
    GC_STAMP(4);
    PST(4);
    pair_barrier();
    PST(5);
    GC_STAMP(5);

    // ---- phase 3 opens: both waves merge the count planes (SW: W0 takes W1's slider sets), W0
    // takes the 3-fold verdict
    if constexpr (SW) {
        if (role == 0) {
            H.cw[1] |= L.swc[0][l];
            H.cw[2] |= L.swc[1][l];
        }
    } else {
#pragma unroll
        for (int b = 0; b < 5; b++) ms.cnt[b] |= L.planes[role ^ 1][b][l];
    }
    ms.total = part + (int)L.part[role ^ 1][l];  // W0's part holds the castles
    if (role == 0) {
        u32 rpk = L.rep[l];
        c = (int)(rpk & 0xFFu);
        hl = rpk >> 8;
    }
    H.ns = ns;
    H.mr = mr;
    H.irrev = irrev;
    H.my_chk = my_chk;
    H.opp_chk = opp_chk;
    H.both = both;
    H.mv = mv;
    H.c = c;
    H.hl = hl;
    H.ep_from = ep_from;
    H.ep = ep;
}

// env_ply's epilogue (gc_env.h): the post-move board with the check flags of both sides, the
// window length and M_DONE when the pre-move board reached 3 occurrences or the window is full
__device__ __forceinline__ Pos pair_settle(const PairHalf& H, bool white) {
    u32 chk = white ? ((H.my_chk ? M_WCHK : 0u) | (H.opp_chk ? M_BCHK : 0u))
                    : ((H.opp_chk ? M_WCHK : 0u) | (H.my_chk ? M_BCHK : 0u));
    Pos ns = H.ns;
    ns.meta = with_hl((ns.meta & ~(u32)(M_WCHK | M_BCHK | M_DONE)) | chk | ((H.c >= 3 || H.c == 0) ? M_DONE : 0u), H.hl);
    return ns;
}

// The self-play pick from the move sets in LDS (pair_half with SW): the set holding rank k by
// the byte counts (gc_core.h sw_locate), then that one set from LDS; more moves than byte sums
// hold (never in play) take a rolled scan over LDS.  k < tot.
template <class LdsT>
__device__ __forceinline__ int sw_pick_lds(const LdsT& L, int l, const Gen& g, const u64* cw, int tot, int k) {
    const int normal = tot - popc(g.castles);
    int r = k, j;
    if (tot < 256) {
        j = sw_locate(cw, r);
    } else {
#pragma unroll 1
        for (j = 0; j < SW_SETS - 1; j++) {
            const int c = popc(L.sets[j][l]);
            if (r < c) break;
            r -= c;
        }
    }
    j = j < SW_SETS ? j : SW_SETS - 1;  // a castle's rank runs past the sets
    const int set_act = sw_finish(g, j, L.sets[j][l], r);
    return k >= normal ? sw_castle(g, k - normal) : set_act;
}

// One ply of the paired driver (opponent "none").  In/out: the state s, the action a (picked
// for s by the previous ply or by the reset), the draw counter d (W0), the window h (W1; its
// table write is left deferred in h), the step counter nst.  Returns the ply's env.step()
// outputs; on return both waves hold the same s, and with SHARE_ACT the same next action a
// (W0 picks it; it crosses to W1 through LDS).
template <bool SHARE_ACT, bool FIDE = false, class RT = int>
__device__ __forceinline__ StepOut pair_ply(PairLds& L, const PairCtx& C, RT role, int l, int i,
                                            bool live, const Pos& rp, Pos& s, int& a, u32& d, DevHist& h,
                                            u32& nst) {
    constexpr bool SW = true;  // the self-play policy's move-set order (gc_core.h sw_*), both rule sets
    const bool none = a == A_NONE;                           // empty list: driver reset
    const bool done0 = (s.meta & M_DONE) != 0;               // chess_v2.py:245-251
    const bool cap = mc_of(s.meta) > MOVES_MAX;              // 252-258
    const bool mv = live && !none && !done0 && !cap;         // env_ply runs
    const bool white = (s.meta & M_WHITE) != 0;
    u32 x0 = 0;
    uint16_t ra = (uint16_t)A_NONE;
    PairHalf H;
    // W1, phase 0: the Philox word of the next draw and, for a board that resets this ply,
    // its pick from the start position's table (a serial multiply chain and a load, hidden
    // behind W0's move; the table read lands long before phase 3)
    pair_half<FIDE, false, false, SW>(
        L, role, l, mv, false, s, a, nullptr, nullptr, h, H,
        [&] {
            x0 = philox_x0(C.seed, (u32)i, d);  // the next draw (independent of the position)
            if (C.rtable) ra = C.racts[scale_rank(x0, C.rtotal)];
            L.x0[l] = x0;
        },
        [&] { L.ra[l] = ra; });
    if (role == 0) {
        x0 = L.x0[l];
        ra = (uint16_t)L.ra[l];
    }
    else h.commit();  // the window write, issued before the outcome (not with the stores: 9.3 -> 9.1 us per ply)
    Gen& g = H.g;
    MoveSet& ms = H.ms;
    // W0: the next action from this ply's move sets, ahead of the outcome (its LDS read and rank
    // arithmetic overlap the outcome's; used unless the board resets)
    int set_act = A_NONE;
    if (role == 0 && ms.total > 0) set_act = sw_pick_lds(L, l, g, H.cw, ms.total, (int)scale_rank(x0, (u32)ms.total));
    StepOut o = {0, 0, R_NONE, 0};
    bool have = false;
    if (none) {
        o.reason = R_NO_MOVES;
    } else {
        nst += 1;
        if (done0) { o.done = 1; o.reason = R_DONE_ALREADY; }
        else if (cap) { o.done = 1; o.reason = R_MOVE_CAP; }
        else if (H.both) { o.done = 1; o.reason = R_BOTH_CHECKED; }
        else {
            s = pair_settle(H, white);
            o.reward = -10 + H.mr;
            o.moved = 1;
            if (H.c >= 3) { o.done = 1; o.reason = R_REPETITION; }  // chess_v2.py:404-407
            if (H.c == 0) { o.done = 1; o.reason = R_WINDOW_FULL; }
            if (ms.total == 0 && H.opp_chk) {  // 270-272
                s.meta |= M_DONE;
                o.done = 1;
                o.reward += 100;
                o.reason = R_MATE;
            }
            if (!o.done && !white) s.meta += (1u << M_MC_SHIFT);  // 291-292
            have = true;
        }
        if (o.done) have = false;
    }
    if (!have) {  // reset (chess_v2.py:183-206), also the no-move driver reset
        s = rp;
        h.bump_gen();
    }
    if (role == 0) {
        uint16_t act = (uint16_t)set_act;
        int tot = ms.total;
        if (!have && C.rtable) {  // the start position's table
            act = ra;
            tot = (int)C.rtotal;
        } else if (!have) {  // the start position without a table (rare): generated, through LDS
            if constexpr (FIDE) {
                gcf::FGen fr;
                gcf::fgen(s, fr);
                g = fr.g;
                tot = gcf::fsw_gen(s, fr, H.T);
            } else {
                gen_init(s, g);
                tot = sw_gen(s, g, H.T);
            }
            H.cw[0] = H.cw[1] = H.cw[2] = H.cw[3] = 0;
            sw_pack(H.T, 0, SW_SETS, H.cw);
#pragma unroll
            for (int j = 0; j < SW_SETS; j++) L.sets[j][l] = H.T[j];
            act = (uint16_t)(tot > 0 ? sw_pick_lds(L, l, g, H.cw, tot, (int)scale_rank(x0, (u32)tot)) : A_NONE);
        }
        a = act;
        d += tot > 0 ? 1u : 0u;
        if (SHARE_ACT) {
            L.act[l] = act;
            L.draw[l] = d;
        }
    }
    if (SHARE_ACT) {  // the next action and draw counter to W1; LDS free for the next ply
        PST(6);
        pair_barrier();
        PST(7);
        if (role) {
            a = (int)L.act[l];
            d = L.draw[l];
        }
    }
    return o;
}

// ----------------------------------------------------------------------------- paired step, opponent "random"
// One step() with the random opponent (chess_v2.py:219-294 with opponent_policy set; gc_env.h
// env_step_vs / env_open_vs; the one-wave k_env_step<true, true>) on the paired driver: the
// agent's half-ply, the opponent's reply, and -- for a BLACK agent whose env resets -- the
// opponent's opening, each one pair_half.  The draws of one step come from the same Philox
// stream in the same order as the one-wave kernel: reply (d), [opening], the agent's next
// pick; W1 computes the words of d, d+1 (, d+2) and the start-position-table picks of d and
// d+1 in phase 0 of the agent's half-ply, before it knows which it needs.
// Used when the start position has a pick table and (BLACK) no opening of it can leave
// both kings in check (InitCache::open_safe); otherwise the one-wave kernel runs.
struct PairLdsVs : PairLds {
    u32 x1[PAIR_BOARDS];  // W1 -> W0: the Philox words of draws d+1, d+2
    u32 x2[PAIR_BOARDS];
    u32 oa[PAIR_BOARDS];  // W0 -> W1: the opponent's reply (read in its phase 1)
    u32 vote[2];          // per wave: some board of it resets (BLACK: the opening half-ply runs)
};

template <bool BLACK, bool SHARE_ACT, class RT = int>
__device__ __forceinline__ StepOut pair_step_vs(PairLdsVs* Ls, PairLdsVs& L, const PairCtx& C, RT role, int l,
                                                int i, bool live, const Pos& rp, Pos& s, int& a, u32& d, DevHist& h,
                                                u32& nst) {
    const bool none = a == A_NONE;                           // empty list: driver reset
    const bool done0 = (s.meta & M_DONE) != 0;               // chess_v2.py:245-251
    const bool cap = mc_of(s.meta) > MOVES_MAX;              // 252-258
    const bool mv = live && !none && !done0 && !cap;         // the agent's ply runs
    const bool white = (s.meta & M_WHITE) != 0;              // the agent's colour
    u32 x0 = 0, x1 = 0, x2 = 0, ra = 0;
    PairHalf H;
    // ---- the agent's half-ply (every half-ply generates set-wise: the picks are in move-set order)
    pair_half<false, false, false, true>(
        L, role, l, mv, false, s, a, nullptr, nullptr, h, H,
        [&] {
            x0 = philox_x0(C.seed, (u32)i, d);
            x1 = philox_x0(C.seed, (u32)i, d + 1);
            if (BLACK) x2 = philox_x0(C.seed, (u32)i, d + 2);
            ra = (u32)C.racts[scale_rank(x0, C.rtotal)] | ((u32)C.racts[scale_rank(x1, C.rtotal)] << 16);
            L.x0[l] = x0;
            L.x1[l] = x1;
            if (BLACK) L.x2[l] = x2;
        },
        [&] { L.ra[l] = ra; });
    if (role == 0) {
        x0 = L.x0[l];
        x1 = L.x1[l];
        if (BLACK) x2 = L.x2[l];
    }
    ra = L.ra[l];  // W1 wrote it before the barrier that closed phase 2
    StepOut o = {0, 0, R_NONE, 0};
    bool cont = false;  // the opponent replies
    if (none) {
        o.reason = R_NO_MOVES;
    } else {
        nst += 1;
        if (done0) { o.done = 1; o.reason = R_DONE_ALREADY; }
        else if (cap) { o.done = 1; o.reason = R_MOVE_CAP; }
        else if (H.both) { o.done = 1; o.reason = R_BOTH_CHECKED; }
        else {
            s = pair_settle(H, white);
            o.reward = -10 + H.mr;
            o.moved = 1;
            if (H.c >= 3) { o.done = 1; o.reason = R_REPETITION; }
            if (H.c == 0) { o.done = 1; o.reason = R_WINDOW_FULL; }
            if (H.ms.total == 0 && H.opp_chk) {  // 270-272
                s.meta |= M_DONE;
                o.done = 1;
                o.reward += 100;
                o.reason = R_MATE;
            }
            if (!o.done && H.ms.total == 0) {  // 120-122: the opponent "resigns"
                s.meta |= M_DONE;
                o.done = 1;
                o.reason = R_OPP_NO_MOVE;
            }
            cont = !o.done;
        }
    }
    int nd = cont ? 1 : 0;  // draws taken so far this step
    // ---- the opponent's reply: W0 picks it from the agent ply's generation (draw d)
    int oa = A_NONE;  // W1 reads W0's pick in the reply's phase 1
    if (role == 0) {
        if (cont) oa = sw_pick_lds(L, l, H.g, H.cw, H.ms.total, (int)scale_rank(x0, (u32)H.ms.total));
        L.oa[l] = (u32)oa;
    } else if (live) {
        h.commit();  // the agent ply's window write lands before the reply probes the table
    }
    const Pos s1 = s;
    pair_half<false, true, false, true>(L, role, l, cont, false, s1, oa, L.oa, nullptr, h, H, PairNoop{}, PairNoop{});
    if (cont) {
        if (H.both) {
            o.reason = R_BOTH_CHECKED;
            o.done = 1;
        } else {
            s = pair_settle(H, !white);
            o.reward -= H.mr;  // 283
            if (H.c >= 3) { o.done = 1; o.reason = R_REPETITION; }
            if (H.c == 0) { o.done = 1; o.reason = R_WINDOW_FULL; }
            if (H.ms.total == 0 && H.opp_chk) {  // 285-288
                s.meta |= M_DONE;
                o.done = 1;
                o.reward -= 100;
                o.reason = R_MATED;
            }
            if (s.meta & M_WHITE) s.meta += (1u << M_MC_SHIFT);  // 291-292
        }
    }
    const bool have = o.moved && !o.done;
    if (!have) {  // reset (chess_v2.py:183-206), also the no-move driver reset
        s = rp;
        h.bump_gen();
    }
    // ---- the agent's next action (W0): from the reply's generation, or the start position's table
    uint16_t act = (uint16_t)A_NONE;
    int tot = 0;
    if (role == 0) {
        if (have) {
            tot = H.ms.total;
            if (tot > 0) act = (uint16_t)sw_pick_lds(L, l, H.g, H.cw, tot, (int)scale_rank(x1, (u32)tot));
        } else if (!BLACK) {
            tot = (int)C.rtotal;
            act = (uint16_t)(nd ? ra >> 16 : ra & 0xFFFFu);
        }
    }
    if constexpr (BLACK) {
        // ---- the opponent's opening after a reset (env_open_vs), when some board of the
        // workgroup needs it: its pick from the table (draw d + nd), one half-ply, its 3-fold
        // verdict discarded, move_count 1; then the agent's pick from its generation
        const bool open = live && !have;
        const unsigned long long vote = __ballot(open);
        if (l == 0) L.vote[role] = vote != 0 ? 1u : 0u;
        if (role) {
            if (live) h.commit();
        }
        pair_barrier();
        bool any = false;
#pragma unroll
        for (int q = 0; q < PAIRS_WG; q++) any = any || Ls[q].vote[0] != 0 || Ls[q].vote[1] != 0;
        if (any) {
            const int oa = (int)(nd ? ra >> 16 : ra & 0xFFFFu);
            const Pos s0 = s;
            pair_half<false, false, false, true>(L, role, l, open, false, s0, oa, nullptr, nullptr, h, H, PairNoop{},
                                                 PairNoop{});
            if (open) {
                s = pair_settle(H, true);
                s.meta = (s.meta & ~(u32)M_DONE) + (1u << M_MC_SHIFT);
                nd += 1;
                if (role == 0) {
                    tot = H.ms.total;
                    act = (uint16_t)A_NONE;
                    if (tot > 0)
                        act = (uint16_t)sw_pick_lds(L, l, H.g, H.cw, tot, (int)scale_rank(nd == 1 ? x1 : x2, (u32)tot));
                }
            }
        }
    }
    if (role == 0) {
        a = act;
        d += (u32)nd + (tot > 0 ? 1u : 0u);
        if (SHARE_ACT) {
            L.act[l] = act;
            L.draw[l] = d;
        }
    }
    if (SHARE_ACT) {  // the next action and draw counter to W1; LDS free for the next step
        pair_barrier();
        if (role) {
            a = (int)L.act[l];
            d = L.draw[l];
        }
    }
    return o;
}

// entry loads of the paired kernels (both waves load every input: a role branch that loads
// into a register on one side and zeroes it on the other makes the compiler drain every
// outstanding load before the zeroing)
struct PairIO {
    u64* bb; u32* meta; u32* hgen; u32* draw; u32* nsteps; int32_t* reward; uint16_t* act; uint8_t* done;
    uint8_t* reason; int n;
    __device__ PairIO(uint8_t* slab, int nn)
        : bb(reinterpret_cast<u64*>(slab)), meta(reinterpret_cast<u32*>(slab + Slab::meta(nn))),
          hgen(reinterpret_cast<u32*>(slab + Slab::hgen(nn))), draw(reinterpret_cast<u32*>(slab + Slab::draw(nn))),
          nsteps(reinterpret_cast<u32*>(slab + Slab::nsteps(nn))),
          reward(reinterpret_cast<int32_t*>(slab + Slab::reward(nn))),
          act(reinterpret_cast<uint16_t*>(slab + Slab::act(nn))), done(slab + Slab::done(nn)),
          reason(slab + Slab::reason(nn)), n(nn) {}
    __device__ Pos load(int i) const {
        size_t N = (size_t)n;
        Pos s;
        s.k = bb[i]; s.q = bb[N + i]; s.r = bb[2 * N + i]; s.b = bb[3 * N + i];
        s.n = bb[4 * N + i]; s.p = bb[5 * N + i]; s.w = bb[6 * N + i];
        s.meta = meta[i];
        return s;
    }
    __device__ void store(int i, const Pos& s) const {
        size_t N = (size_t)n;
        bb[i] = s.k; bb[N + i] = s.q; bb[2 * N + i] = s.r; bb[3 * N + i] = s.b;
        bb[4 * N + i] = s.n; bb[5 * N + i] = s.p; bb[6 * N + i] = s.w;
        meta[i] = s.meta;
    }
};

// The store pointers, re-derived at the end of the kernel from an opaque copy of n: left to
// CSE, the entry pointers (18 SGPRs) would stay live through the whole ply and push the
// compiler into SGPR spills.
__device__ __forceinline__ PairIO store_io(uint8_t* slab, int nn) {
    asm volatile("" : "+s"(nn));
    return PairIO(slab, nn);
}

// The paired kernels take no EnvDev: every argument fits the 16 preloaded dwords
// (hipcc -mllvm -amdgpu-kernarg-preload-count=16; step: 13, rollout: 16), which arrive in
// SGPRs at wave launch.  A kernel-argument s_load is a round trip to the kernarg buffer at
// every launch -- measured ~2-3k cycles, paid wherever the compiler sinks it, and with SGPRs
// scarce it sank it next to a spill that forced the wait in phase 1.  The reset position and
// move set come from a device-memory copy (icd) instead.
// Which pair and role wave w of a workgroup takes: pair w / 2, the role alternating across pairs
// (a SIMD hosts both roles).  r03 A/B (fused, 65 536 boards): 11.37e9; a pair's waves as roles
// 0 / 1 everywhere 11.2e9; waves w and w + 4 (one SIMD) as a pair with 4 pairs 10.9e9.
__device__ __forceinline__ int pair_of_wave(int w) { return w >> 1; }
__device__ __forceinline__ int role_of_wave(int w) { return (w ^ (w >> 1)) & 1; }
#define PAIR_PROLOGUE PAIR_PROLOGUE_ACT(in_io.act, )
// ACTS: the action source (the env's next action, or the caller's for the API step);
// ENTRY: more entry loads, waited for with the reset position's
#define PAIR_PROLOGUE_ACT(ACTS, ENTRY)                                                                      \
    using LdsT = typename std::conditional<OPP != 0 || API, PairLdsVs, PairLds>::type;                      \
    __shared__ LdsT Ls[PAIRS_WG];                                                                           \
    const int wv_ = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); /* wave-uniform */            \
    const int pw = PAIRS_WG > 1 ? pair_of_wave(wv_) : 0;                                                    \
    LdsT& L = Ls[pw];                                                                                       \
    const int role = role_of_wave(wv_);                                                                     \
    const int l = threadIdx.x & (PAIR_BOARDS - 1);                                                          \
    const int blk = blockIdx.x * PAIRS_WG + pw + blk0; /* board block (a launch may cover a sub-range) */   \
    const int i = blk * PAIR_BOARDS + l;                                                                    \
    const bool live = i < nn;                                                                               \
    const int ii = live ? i : nn - 1; /* dead lanes read a valid board, store nothing */                    \
    const PairIO in_io(slab, nn);                                                                           \
    const PairCtx C = {seed, htab, in_io.hgen, racts, icd, (rinfo >> 16) != 0, rinfo & 0xFFFFu};                 \
    GC_STAMP(0);                                                                                            \
    Pos s = in_io.load(ii);                                                                                 \
    u32 ua = ACTS[ii], g0 = in_io.hgen[ii], nst = in_io.nsteps[ii], d = in_io.draw[ii];                     \
    /* the reset position (HBM, scalar loads): waited for only after the board loads above have */         \
    /* issued (an asm use is a scheduling barrier for memory operations: placed first, its round */        \
    /* trip delayed every global load); the opaque use keeps it from being re-loaded at the reset */       \
    Pos rp = icd->pos;                                                                                      \
    asm volatile("" : "+v"(rp.k), "+v"(rp.q), "+v"(rp.r), "+v"(rp.b), "+v"(rp.n), "+v"(rp.p), "+v"(rp.w),  \
                 "+v"(rp.meta)); /* VGPRs: SGPRs are the scarce file here */                                  \
    ENTRY                                                                                                   \
    pin(s); pin(ua); pin(g0); pin(nst); pin(d);                                                             \
    GC_STAMP(1);                                                                                            \
    int a = (int)ua;                                                                                        \
    DevHist h = DevHist{htab, in_io.hgen, g0, ii, OPP == 2 ? HTAB_BITS_UNCAPPED : HTAB_BITS};                \
    if constexpr (OPP == 2) h.sp = icd->spill; /* a BLACK agent's windows may spill */

// One step of the paired driver: opponent "none" (OPP 0: pair_ply) or the random opponent
// with a WHITE (1) or BLACK (2) agent (pair_step_vs).
template <int OPP, bool SHARE_ACT, bool FIDE, class LdsT, class RT>
__device__ __forceinline__ StepOut pair_step(LdsT* Ls, LdsT& L, const PairCtx& C, RT role, int l, int i, bool live,
                                             const Pos& rp, Pos& s, int& a, u32& d, DevHist& h, u32& nst) {
    if constexpr (OPP == 0) return pair_ply<SHARE_ACT, FIDE, RT>(L, C, role, l, i, live, rp, s, a, d, h, nst);
    else return pair_step_vs<OPP == 2, SHARE_ACT, RT>(Ls, L, C, role, l, i, live, rp, s, a, d, h, nst);
}

template <bool FIDE, int OPP = 0>
__global__ void __launch_bounds__(2 * PAIR_BOARDS * PAIRS_WG) PAIR_ATTR
    k_env_step2(uint8_t* __restrict__ slab, int nn, int blk0, uint64_t seed, u64* __restrict__ htab,
                const uint16_t* __restrict__ racts, const EnvDev::InitCache* __restrict__ icd,
                u32 rinfo /* ic.table << 16 | ic.total */) {
    constexpr bool API = false;
    PAIR_PROLOGUE
    StepOut o = pair_step<OPP, false, FIDE>(Ls, L, C, role, l, i, live, rp, s, a, d, h, nst);
    GC_STAMP(6);
    const PairIO io = store_io(slab, nn);
    if (live) {
        if (role == 0) {
            io.act[i] = (uint16_t)a;
            io.draw[i] = d;
        } else {
            h.commit();
            io.store(i, s);
            h.flush(g0);
            io.nsteps[i] = nst;
            io.reward[i] = o.reward;
            io.done[i] = (uint8_t)o.done;
            io.reason[i] = (uint8_t)o.reason;
        }
    }
    GC_STAMP(7);
#ifdef GC_STAMPS
    if (g_stamp_out != nullptr && l == 0)
        for (int q = 0; q < 8; q++) g_stamp_out[((size_t)blk * 2 + role) * 8 + q] = gc_stamp_lds[threadIdx.x >> 6][q];
#endif
}


// One ply's env.step() outputs, packed for the per-ply trace [ply][N] (one coalesced 8-B
// store per board per ply): action played (int16; -1 = none, the driver's no-move reset),
// reward (int16), done (u8), reason (u8).  Unpacked by gc_env_rollout / bench consumers.
__device__ __forceinline__ u64 trace_word(int played, const StepOut& o) {
    return (u64)(uint16_t)(int16_t)played | ((u64)(uint16_t)(int16_t)o.reward << 16) | ((u64)(o.done & 0xFF) << 32) |
           ((u64)(o.reason & 0xFF) << 40);
}
#define ROLLOUT_MAX_PLIES 16383  // plies per launch: rinfo bits 18..31

#ifdef GC_PSTAMPS
// the wave's start (s_memrealtime) with its placement in bits 44+: cu | sh | se | simd | xcc
// (tools/pstamp_probe.py splits them; as GC_STAMPS_REAL)
__device__ __forceinline__ unsigned long long pst_entry_where() {
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)\n\ts_getreg_b32 %1, hwreg(HW_REG_XCC_ID)" : "=s"(hw), "=s"(xcc));
    const unsigned long long where = ((hw >> 8) & 0xF) | (((hw >> 12) & 1) << 4) | (((hw >> 13) & 3) << 5) |
                                     (((hw >> 4) & 3) << 7) | ((unsigned long long)(xcc & 0xF) << 9);
    return (t & ((1ull << 44) - 1)) | (where << 44);
}
#endif

// Fused K-ply random self-play on the paired step: the state stays in registers for the K
// plies (K env.step() calls of every board in one launch); every ply's outputs go to the
// optional trace [ply][N] (trace_word), the last ply's outputs, the state, window and counters
// and the per-board stats (as k_env_rollout) are written at the end.  rinfo = plies << 18 |
// ic.table << 16 | ic.total: with the trace pointer, all 16 argument dwords are preloaded.
template <bool FIDE, int OPP = 0>
__global__ void __launch_bounds__(2 * PAIR_BOARDS * PAIRS_WG) PAIR_ATTR
    k_env_rollout2(uint8_t* __restrict__ slab, int nn, uint64_t seed, u64* __restrict__ htab,
                   const uint16_t* __restrict__ racts, const EnvDev::InitCache* __restrict__ icd, u32 rinfo,
                   uint64_t* __restrict__ stats, u64* __restrict__ trace) {
    constexpr bool API = false;
    constexpr int blk0 = 0;
    const int plies = (int)(rinfo >> 18);
    rinfo &= 0x1FFFFu;
#ifdef GC_PSTAMPS
    const unsigned long long g_pst_entry = pst_entry_where();  // wave start, before the entry loads
#endif
    PAIR_PROLOGUE
    uint64_t steps = 0, rsum = 0;
    u32 e_mate = 0, e_rep = 0, e_cap = 0, e_nomove = 0, e_err = 0;
    StepOut o = {0, 0, R_NONE, 0};
#ifdef GC_PSTAMPS
    unsigned long long rt0 = 0, rt1 = 0;  // 100 MHz wall clock: after the entry loads, after the first ply
    if (l == 0) {
        for (int k = 0; k < 8; k++) gc_pst[threadIdx.x >> 6][k] = 0;
        gc_pst[threadIdx.x >> 6][8] = __builtin_amdgcn_s_memtime();
    }
    rt0 = __builtin_amdgcn_s_memrealtime();
#endif
    // one loop per role (RoleC): each wave runs only its own role's code; and one with the
    // per-board stats (gc_env_rollout), one without (the device form: no counters per ply)
    // a CU's two workgroups take turns one priority level up, ply by ply (k_env_rollout4's
    // GC_WG_FAIR: blocks b and b + half; at equal priority the SQ issues the older wave first)
    const int wg_half = ((nn + PAIR_BOARDS * PAIRS_WG - 1) / (PAIR_BOARDS * PAIRS_WG)) >> 1;
    auto plies_loop = [&](auto R, auto ST) {
        for (int p = 0; p < plies; p++) {
            int played = a;
            if (GC_PAIR_FAIR) {
                if ((((int)blockIdx.x >= wg_half) ? 1 : 0) ^ (p & 1)) __builtin_amdgcn_s_setprio(1);
                else __builtin_amdgcn_s_setprio(0);
            }
            o = pair_step<OPP, true, FIDE>(Ls, L, C, R, l, i, live, rp, s, a, d, h, nst);
#ifdef GC_PSTAMPS
            if (p == 0) rt1 = __builtin_amdgcn_s_memrealtime();
#endif
            if (R) {  // W1: the ply's outputs (trace, stats) and the window write
                if (trace && live) trace[(size_t)p * nn + i] = trace_word(played == A_NONE ? -1 : played, o);
                if (!ST) {
                } else if (played == A_NONE) {
                    e_nomove++;
                } else {
                    steps++;
                    rsum += (uint64_t)(int64_t)o.reward;
                    if (o.done) {
                        e_mate += o.reason == R_MATE || o.reason == R_MATED;
                        e_rep += o.reason == R_REPETITION;
                        e_cap += o.reason == R_MOVE_CAP;
                        e_err += o.reason == R_BOTH_CHECKED || o.reason == R_WINDOW_FULL;
                        e_nomove += o.reason == R_OPP_NO_MOVE;
                    }
                }
                h.commit();  // this ply's window write lands before the next ply's probe
            }
        }
        // the launch's end (in the role's own code: nothing of the other role's state stays live)
#ifdef GC_PSTAMPS
        if (g_pst_out != nullptr && l == 0) {
            const size_t w = (size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
            for (int k = 0; k < 8; k++) g_pst_out[w * 12 + k] = gc_pst[threadIdx.x >> 6][k];
            g_pst_out[w * 12 + 8] = g_pst_entry;  // (set below)
            g_pst_out[w * 12 + 9] = rt0;
            g_pst_out[w * 12 + 10] = rt1;
            g_pst_out[w * 12 + 11] = __builtin_amdgcn_s_memrealtime();
        }
#endif
        const PairIO io = store_io(slab, nn);
        if (live) {
            if (R == 0) {
                io.act[i] = (uint16_t)a;
                io.draw[i] = d;
            } else {
                io.store(i, s);
                h.flush(g0);
                io.nsteps[i] = nst;
                io.reward[i] = o.reward;
                io.done[i] = (uint8_t)o.done;
                io.reason[i] = (uint8_t)o.reason;
                if (ST) {
                    uint64_t* so = stats + 8 * (size_t)i;
                    so[0] += steps; so[1] += rsum;
                    so[2 + R_MATE] += e_mate; so[2 + R_REPETITION] += e_rep; so[2 + R_MOVE_CAP] += e_cap;
                    so[2 + R_NO_MOVES] += e_nomove; so[2 + R_BOTH_CHECKED] += e_err;
                }
            }
        }
    };
    if (role == 0) plies_loop(RoleC<0>{}, std::false_type{});  // W0 keeps no stats (one loop for
    else if (stats) plies_loop(RoleC<1>{}, std::true_type{});  // both roles: 965 -> 1 045 VALU per wave)
    else plies_loop(RoleC<1>{}, std::false_type{});
}

// ----------------------------------------------------------------------------- quad step
// k_env_rollout4: the headline rollout (opponent "none", reference rules, move-set order) with
// FOUR waves per 64 boards.  With two (k_env_rollout2) a SIMD holds 2 waves -- all 65 536
// boards give -- and a wave's ply is one long dependency chain: a lone wave runs its ply in
// 3.75 us, two share the SIMD at 6.0 us each (tools/pstamp_probe.py), VALU issue ~35 % busy.
// The ply's parallel parts -- the enemy map's three parts, the own slider sets' two halves --
// go to their own waves, so each wave's chain is shorter and a SIMD holds four of them:
//
//   phase 0   Q0: applies the action (the last ply's pick) -> post-move board to LDS
//             Q1: the Philox word, the reset table read (its window probe is in flight)
//   phase 1   Q0: checkers, check mask, pins                   Q1: the mover's own check flag
//             Q2: enemy leaper + orthogonal slider attacks     Q3: enemy diagonal slider attacks
//   phase 2   Q0: castles, pawn and knight sets                Q1: the 3-fold commit
//             Q2: the own rook/queen direction sets, king sets Q3: the bishop/queen ones
//   phase 3   Q0: the outcome                                  Q1: the outcome, the stores, the
//             Q2: the pick of the next action                      next ply's window probe
//
// Q0 and Q1 carry the board's state between plies; Q2 and Q3 are stateless (the post-move
// board and the pins come through LDS) and compute their sets unconditionally -- ignored,
// like the totals, when no generation is due.  Same decisions in the same order as
// pair_ply (and so as k_env_step<true, false> and the oracle): tests/test_gpu_parity.py and
// tests/test_full_size.py run the fused rollouts against the oracle and the launched kernel.
#define QUAD_BOARDS 64
#ifndef QUADS_WG
#define QUADS_WG 2  // two quads per workgroup; the second's roles rotated by 2 so that every SIMD
                    // hosts a state-carrying and a stateless role of each workgroup
#endif
// The 3-fold window's occupancy in LDS (k_env_rollout4<true>; Q1's, a bit per table slot: 64 B per board).
// The table is open-addressed with linear probing and entries leave it only all at once (a
// generation bump), so a board whose home slot is free is not in the window -- its probe would
// stop at once and insert there.  While a board's bitmap mirrors its window (OccQ::valid: since the
// window was last emptied inside this launch -- a reset or an irreversible move), Q1 tests the
// next board's home slot in LDS and loads nothing when it is free (~80 % of plies: the window is
// short and a repetition is rare); a taken home slot (the board again, or another on its slot)
// is probed in the table as before, and so is every board of a window that predates the launch.
// Exact: the fast path makes the same decision rep_commit makes on a free first probe.  It
// removes the probe's line from most plies (the window's bytes).  Where the
// work goes (tools/pstamp_probe.py: the ply's chain is Q2's, phases 1-3): the bitmap is cleared
// and the next board looked up in phase 1 (Q1 computes only the mover's check flag there), this
// ply's entry is added in phase 2 beside the commit; in phase 3 every lane issues ONE load as
// before -- a slow lane its home entry, a fast lane the env's init block, one line that every
// lane of the chip reads (it stays in L2) -- so the registers merge no loaded data and the wait
// stays at phase 2's commit; the fast lane's header is replaced after it.  (v1, all of it in
// phase 3: Q1's phase 3 2 589 vs 1 447 cycles, -5 % at K = 1 000; v2, a load issued only by the
// slow lanes: the merge of the loaded registers waited for it at the end of phase 3.)

struct QuadLds {
    u64 sets[SW_SETS][QUAD_BOARDS];  // the next side's move sets (Q0: pawns / knights, Q2, Q3)
    u64 ns[NBB][QUAD_BOARDS];        // Q0 -> all: the post-move board (phase 0)
    u32 nmeta[QUAD_BOARDS];
    int32_t mr[QUAD_BOARDS];         //           its capture reward
    u32 irrev[QUAD_BOARDS];          //           irreversible move
    u64 pin3[3][QUAD_BOARDS];        // Q0 -> Q2, Q3: check mask, pinned, pin rays
    u32 f0[QUAD_BOARDS];             // Q0 -> Q1: the side to move is in check
    u64 enemy[3][QUAD_BOARDS];       // Q2 / Q3 -> Q0, Q2: the enemy map's leaper + orthogonal ([1]), diagonal ([2]) parts
    u32 f1[QUAD_BOARDS];             // Q1 -> Q0: the mover is in check after its move
    u64 cwx[2][4][QUAD_BOARDS];      // Q2 ([0]) / Q3 ([1]) -> Q2: their sets' byte counts (all four words)
    u64 cw0[2][QUAD_BOARDS];         // Q0 -> Q2: its sets' byte counts (words 0, 1: pawns, knights)
    u32 part[4][QUAD_BOARDS];        // partial move totals (Q0's holds the castles)
    u32 rep[QUAD_BOARDS];            // Q1 -> Q0: 3-fold count | window length << 8
    u32 x0[QUAD_BOARDS];             // Q1 -> Q2: the Philox word of the next draw
    u32 ra[QUAD_BOARDS];             // Q1 -> Q0: the start-position table pick
    u32 act[QUAD_BOARDS];            // Q0 -> Q1: this ply's action (phase 0)
    u32 pick[QUAD_BOARDS];           // Q2 -> Q0: the policy's pick from this ply's move sets (phase 3)
    u32 castles[QUAD_BOARDS];        // Q0 -> Q2: the castles (phase 2)
    u64 occ[HTAB / 64][QUAD_BOARDS];  // (OCC) Q1: the window's taken table slots, a bit per slot
    u32 nkey[QUAD_BOARDS];            // (OCC) Q1, phase 1 -> 3: the next board's key if the move stands
    u32 rkey0;                        // (OCC) the reset position's key
    Pos rp;                          // the reset position (read at a reset: no registers held for it)
};
// one set of the next side's moves into LDS, its count into the packed byte counts and the total
template <class LT>
struct QuadSetsT {
    LT& L;
    int l;
    u64 cw[4];
    int part;
    __device__ void put(int j, u64 t) {
        L.sets[j][l] = t;
        const int c = popc(t);
        cw[j >> 3] |= (u64)c << (8 * (j & 7));
        part += c;
    }
    template <int LO, int HI>
    __device__ void put_all(const u64* t) {
#pragma unroll
        for (int j = LO; j < HI; j++) put(j, t[j - LO]);
    }
};
using QuadSets = QuadSetsT<QuadLds>;

// Q0's choice of the next action, left for the start of the next ply: Q2 makes the pick from
// the move sets in phase 3 while Q0 and Q1 settle the outcome (the pick was phase 3's longest
// chain); a board that resets takes the start position's table pick instead.
struct QuadPend {
    bool pending;  // false: `a` is already the action (the launch's first ply)
    bool have;     // the move stood: Q2's pick
    uint16_t ra;   // else: the table pick
    __device__ int resolve(const QuadLds& L, int l, int a) const {
        return !pending ? a : have ? (int)L.pick[l] : (int)ra;
    }
};

// One ply of board i for role R of its quad (RoleC<0..3>).  Q0 / Q1: in/out as pair_ply (s, a,
// d, h, nst); both return the same s and a.  Q2 / Q3: s, a, d, h, nst unused.  oq (Q1, OCC):
// the occupancy bitmap mirrors the window (valid), and is to be cleared before use (clr: a reset)
struct OccQ {
    bool valid;  // the bitmap mirrors the window
    bool clr;    // it is to be cleared first (the window was emptied: a reset, an irreversible move)
    bool probe;  // the next board, if the move stands, is probed in the table
    bool fast;   // the probe in flight is the init block's line: its header reads as a free slot
};
// The two workgroups of a CU (blocks b and b + half: tools/pstamp_probe.py reads each wave's
// HW_ID) start together on the same SIMDs, and at equal priority the SQ issues the older wave
// first -- so block b ran its plies at 4.21 us and block b + half at 5.01 (every CU; same roles on
// every SIMD), and the launch ended with the later ones.  They take turns instead: for turns of
// GC_TURN_SHIFT (below) plies one workgroup's roles run one level above the other's (s_setprio 3 /
// 1 over 2 / 0).  One-ply turns: 0.14 us apart, the launch 4 858 vs 5 636 us by stamps; same box
// 16.01 vs 15.43e9 at K = 1 000, 13.25 vs 13.19e9 at K = 20 (run_r06p).  (Round 3's feedback form,
// progress words per CU, levelled them too but cost more than it gave.)
#ifndef GC_WG_FAIR
#define GC_WG_FAIR 1  // 0: A/B
#endif
// s_setprio(x), one level up on the plies where this workgroup has its turn (GC_WG_FAIR)
#define QSETPRIO(x, up)                                       \
    do {                                                      \
        if (GC_WG_FAIR && (up)) __builtin_amdgcn_s_setprio((x) + 1); \
        else __builtin_amdgcn_s_setprio(x);                   \
    } while (0)
template <int R, bool OCC>
__device__ __forceinline__ StepOut quad_ply(QuadLds& L, const PairCtx& C, int l, int i, bool live, Pos& s, int& a,
                                            u32& d, DevHist& h, u32& nst, RepProbe& pr, QuadPend& pend, OccQ& oq,
                                            bool up = false) {
    constexpr bool CARRY = R < 2;  // Q0 / Q1 hold the state
    // Q2's pick (phase 3's longest) is raised over Q0's outcome there: 14.43-14.63 -> 14.90-15.12e9
    if (R == 0) QSETPRIO(2, up);
    if (R == 2) QSETPRIO(0, up);
    if (GC_WG_FAIR && R == 1) QSETPRIO(2, up);
    if (GC_WG_FAIR && R == 3) QSETPRIO(0, up);
    if (R == 0) a = pend.resolve(L, l, a);  // the last ply's action: Q2's pick, or the reset table's
    u32 x0 = 0;
    uint16_t ra = (uint16_t)A_NONE;
    if (R == 1) {  // phase 0 work first: it does not depend on the action, which Q1 learns after it
        x0 = philox_x0(C.seed, (u32)i, d);  // the next draw (independent of the position)
        if (C.rtable) ra = C.racts[scale_rank(x0, C.rtotal)];
        L.x0[l] = x0;
    }
    if (R == 0) L.act[l] = (u32)a;
    PST(7);  // (GC_PSTAMPS: the segments as in the paired kernel, phase 0 .. wait D)
    if (R == 1) {
        pair_barrier();  // (Q1's phase 0 is above; it meets the others' barrier A here)
        a = (int)L.act[l];
    }
    const bool none = a == A_NONE;                           // empty list: driver reset
    const bool done0 = (s.meta & M_DONE) != 0;               // chess_v2.py:245-251
    const bool cap = mc_of(s.meta) > MOVES_MAX;              // 252-258
    const bool mv = live && !none && !done0 && !cap;         // env_ply runs
    const bool white = (s.meta & M_WHITE) != 0;
    int mr = 0;
    bool irrev = false;
    Pos ns;
    // ---- phase 0
    if (R == 0) {
        ns = s;
        ns.meta = (ns.meta & ~(u32)M_RIGHTS) | eff_rights(s);  // State::new
        if (mv) apply_legal(ns, white, a, &mr, &irrev);
        L.ns[0][l] = ns.k; L.ns[1][l] = ns.q; L.ns[2][l] = ns.r; L.ns[3][l] = ns.b;
        L.ns[4][l] = ns.n; L.ns[5][l] = ns.p; L.ns[6][l] = ns.w;
        L.nmeta[l] = ns.meta;
        L.mr[l] = mr;
        L.irrev[l] = irrev ? 1u : 0u;
    }
    PST(0);
    if (R != 1) pair_barrier();
    PST(1);
    // ---- phase 1
    Gen g;
    bool my_chk = false;
    if (R != 0) {
        ns.k = L.ns[0][l]; ns.q = L.ns[1][l]; ns.r = L.ns[2][l]; ns.b = L.ns[3][l];
        ns.n = L.ns[4][l]; ns.p = L.ns[5][l]; ns.w = L.ns[6][l];
        ns.meta = L.nmeta[l];
    }
    if (R == 1) {
        mr = L.mr[l];
        irrev = L.irrev[l] != 0;
    }
    gen_base(ns, g);
    if (R == 0) {
        gen_pins(ns, g);
        L.pin3[0][l] = g.checkmask;
        L.pin3[1][l] = g.pinned;
        L.pin3[2][l] = g.pinrays;
        L.f0[l] = g.in_check ? 1u : 0u;
    } else if (R == 1) {
        my_chk = mv && mover_checked(s, ns, white, a);
        L.f1[l] = my_chk ? 1u : 0u;
        if constexpr (OCC) {
        if (oq.clr) {  // the window was emptied
#pragma unroll
            for (int w = 0; w < HTAB / 64; w++) L.occ[w][l] = 0ull;
            oq.clr = false;
        }
        // the next ply's pre-move board if this move stands (ns): its key, and whether its home
        // slot is taken in the window before this ply's entry (phase 2 adds that one)
        const u32 nk = board_key(ns);
        L.nkey[l] = nk;
        oq.probe = !oq.valid || ((L.occ[(nk & (HTAB - 1)) >> 6][l] >> (nk & 63)) & 1) != 0;
        }
    } else if (R == 2) {
        L.enemy[1][l] = g.ks >= 0 ? side_attacks_leapers(ns, !g.white) | side_attacks_orth(ns, !g.white) : 0ull;
    } else {
        L.enemy[2][l] = g.ks >= 0 ? side_attacks_diag(ns, !g.white) : 0ull;
    }
    PST(2);
    pair_barrier();
    PST(3);
    // ---- phase 2
#define QUAD_ENEMY(l) (L.enemy[1][l] | L.enemy[2][l])
    if (R == 0) {
        g.enemy_att = QUAD_ENEMY(l);
        gen_castles(ns, g);  // lib.rs:578-610 with the whole enemy map
        my_chk = L.f1[l] != 0;
    } else if (R == 1) {
        g.in_check = L.f0[l] != 0;
    } else {
        g.checkmask = L.pin3[0][l];
        g.pinned = L.pin3[1][l];
        g.pinrays = L.pin3[2][l];
        if (R == 2) g.enemy_att = QUAD_ENEMY(l);  // for the king sets
    }
    const bool opp_chk = g.in_check;
    const bool both = opp_chk && my_chk;  // lib.rs:1442-1446
    const bool gen = mv && !both;
    QuadSets Q{L, l, {0, 0, 0, 0}, 0};  // sets go to LDS as they are made: no 28-set array held
    int c = 0;
    u32 hl = hl_of(s.meta);
    if (R == 0) {  // pawn sets; castles counted here (phase 2 was Q0's longest: knights to Q3, kings to Q2)
        if (gen) {
            u64 T[SW_SETS];
            sw_pawns(ns, g, T);
            Q.put_all<SW_P1, SW_N>(T + SW_P1);
            // the knight sets here, not on Q3: Q0's SIMDs (Q0 + Q2) are the lighter pair in phase 2
            // (same-box A/B: 14.81 vs 14.59e9 at K = 1 000, 4.62 vs 4.70 us per ply at K = 20)
            sw_knights(ns, g, T);
            Q.put_all<SW_N, SW_ORTH>(T + SW_N);
            Q.part += popc(g.castles);
        }
        L.cw0[0][l] = Q.cw[0];
        L.cw0[1][l] = Q.cw[1];
        L.castles[l] = g.castles;
    } else if (R == 1) {
        if (mv && !both) {
            pin(pr.e0.hdr); pin(pr.e0.k); pin(pr.e0.q); pin(pr.e0.r);
            pin(pr.e0.b); pin(pr.e0.n); pin(pr.e0.p); pin(pr.e0.w);
            if (OCC && oq.fast) pr.e0.hdr = (u64)(h.gen() ^ 1u);  // (after the wait: no loaded register merged)
            c = rep_commit(h, s, pr, hl, irrev);  // table write deferred to h.commit()
            if (!OCC) {
            } else if (irrev) {  // the window is cleared: from the next ply on the bitmap mirrors it again
                oq.valid = true;
                oq.clr = true;
                oq.probe = false;
            } else if (h.wkind == 2) {  // this ply's new entry: its slot, and the next board's home?
                L.occ[h.wpos >> 6][l] |= 1ull << (h.wpos & 63);
                oq.probe = oq.probe || (u32)h.wpos == (L.nkey[l] & (HTAB - 1));
            }
        }
        L.rep[l] = (u32)c | (hl << 8);
        L.ra[l] = ra;
    } else if (R == 2) {  // unconditional: ignored unless generation is due
        u64 T[SW_SETS];
        sw_orth(ns, g, T);
        Q.put_all<SW_ORTH, SW_DIAG>(T + SW_ORTH);
        sw_kings(ns, g, T);
        Q.put_all<SW_K, SW_SETS>(T + SW_K);
        L.part[2][l] = (u32)Q.part;
#pragma unroll
        for (int k = 0; k < 4; k++) L.cwx[0][k][l] = Q.cw[k];
    } else {
        u64 T[SW_SETS];
        sw_diag(ns, g, T);
        Q.put_all<SW_DIAG, SW_K>(T + SW_DIAG);
        L.part[3][l] = (u32)Q.part;
#pragma unroll
        for (int k = 0; k < 4; k++) L.cwx[1][k][l] = Q.cw[k];
    }
    if (R == 0) L.part[0][l] = (u32)Q.part;
    PST(4);
    pair_barrier();
    PST(5);
    // ---- phase 3: the outcome (Q0 and Q1, identical arithmetic); Q2 picks the next action
    // from the move sets (Q0 takes it, or the reset table's, at the start of the next ply)
    StepOut o = {0, 0, R_NONE, 0};
    if (R == 0) QSETPRIO(0, up);
    if (R == 2) QSETPRIO(2, up);
    if (R == 2) {  // (on Q3, whose SIMDs Q1 shares: 12.77-12.98 vs 13.30-13.42e9)
        const int total = (int)L.part[0][l] + Q.part + (int)L.part[3][l];
        u64 cw[4];
#pragma unroll
        for (int k = 0; k < 4; k++) cw[k] = Q.cw[k] | L.cwx[1][k][l];
        cw[0] |= L.cw0[0][l];
        cw[1] |= L.cw0[1][l];
        g.castles = L.castles[l];
        // (a board whose generation is not due reads stale sets here: its pick is not taken)
        L.pick[l] = total > 0 ? (u32)sw_pick_lds(L, l, g, cw, total, (int)scale_rank(L.x0[l], (u32)total)) : (u32)A_NONE;
    }
    if constexpr (CARRY) {
        const int total = gen ? (R == 0 ? Q.part : (int)L.part[0][l]) + (int)L.part[2][l] + (int)L.part[3][l] : 0;
        if (R == 0) {
            const u32 rpk = L.rep[l];
            c = (int)(rpk & 0xFFu);
            hl = rpk >> 8;
            ra = (uint16_t)L.ra[l];
        } else {
            h.commit();  // the window write, issued before the outcome
        }
        bool have = false;
        if (none) {
            o.reason = R_NO_MOVES;
        } else {
            nst += 1;
            if (done0) { o.done = 1; o.reason = R_DONE_ALREADY; }
            else if (cap) { o.done = 1; o.reason = R_MOVE_CAP; }
            else if (both) { o.done = 1; o.reason = R_BOTH_CHECKED; }
            else {
                const u32 chk = white ? ((my_chk ? M_WCHK : 0u) | (opp_chk ? M_BCHK : 0u))
                                      : ((opp_chk ? M_WCHK : 0u) | (my_chk ? M_BCHK : 0u));
                s = ns;
                s.meta = with_hl((ns.meta & ~(u32)(M_WCHK | M_BCHK | M_DONE)) | chk | ((c >= 3 || c == 0) ? M_DONE : 0u), hl);
                o.reward = -10 + mr;
                o.moved = 1;
                if (c >= 3) { o.done = 1; o.reason = R_REPETITION; }  // chess_v2.py:404-407
                if (c == 0) { o.done = 1; o.reason = R_WINDOW_FULL; }
                if (total == 0 && opp_chk) {  // 270-272
                    s.meta |= M_DONE;
                    o.done = 1;
                    o.reward += 100;
                    o.reason = R_MATE;
                }
                if (!o.done && !white) s.meta += (1u << M_MC_SHIFT);  // 291-292
                have = true;
            }
            if (o.done) have = false;
        }
        if (!have) {  // reset (chess_v2.py:183-206), also the no-move driver reset
            s = L.rp;
            h.bump_gen();
        }
        // Q1: the next ply's probe, its pre-move board settled, while Q0 still picks (Q1 waits at
        // the next barrier anyway); after this ply's window write, so it sees it
        if (R == 1 && OCC) {  // (the verdict is phases 1-2's; a reset's window is empty, its bitmap cleared next ply)
            pr.key = have ? L.nkey[l] : L.rkey0;
            if (!have) {
                oq.valid = true;
                oq.clr = true;
            }
            oq.fast = !(live && have && oq.probe);
            // one load per lane: the home entry, or the init block's line (a free slot, see above)
            const ulonglong2* src = oq.fast ? reinterpret_cast<const ulonglong2*>(C.icd)
                                            : reinterpret_cast<const ulonglong2*>(h.htab + h.entry((int)(pr.key & (HTAB - 1))) * 8);
            const ulonglong2 e0 = src[0], e1 = src[1], e2 = src[2], e3 = src[3];
            pr.e0 = RepEntry{e0.x, e0.y, e1.x, e1.y, e2.x, e2.y, e3.x, e3.y};
        } else if (R == 1 && live) {
            rep_prefetch(h, s, pr);
        }
        // the draw counter (both: the quads run only with the start position's pick table, so a
        // reset's pick count is its total) and Q0's pending choice of the next action
        const int tot = have ? total : (int)C.rtotal;
        d += tot > 0 ? 1u : 0u;
        if (R == 0) pend = QuadPend{true, have, ra};
    }
    PST(6);
    pair_barrier();  // Q2's pick to Q0; LDS free for the next ply
    return o;
}

// The quads' LDS (static, shared by the role functions below: a direct reference keeps every
// access a ds_ instruction)
__shared__ QuadLds g_quad_lds[QUADS_WG];

// One role's whole launch (its K plies and its stores), inlined into the kernel's switch on the
// role: a non-inlined function takes generic pointers -- flat memory instructions, which count
// in lgkmcnt too, so every barrier's lgkmcnt(0) waited for the window probe in flight.
template <int RR, bool ST, bool OCC>
__device__ __forceinline__ void quad_run(uint8_t* __restrict__ slab, int nn, uint64_t seed, u64* __restrict__ htab,
                                      const uint16_t* __restrict__ racts, const EnvDev::InitCache* __restrict__ icd,
                                      u32 rinfo, int plies, uint64_t* __restrict__ stats, u64* __restrict__ trace,
                                      int qw, int l, int i) {
    QuadLds& L = g_quad_lds[qw];
    const bool live = i < nn;
    const int ii = live ? i : nn - 1;  // dead lanes read a valid board, store nothing
    const PairIO in_io(slab, nn);
    const PairCtx C = {seed, htab, in_io.hgen, racts, icd, (rinfo >> 16) != 0, rinfo & 0xFFFFu};
    Pos s{};
    u32 ua = 0, g0 = 0, nst = 0, d = 0;
    if (RR < 2) {
        s = in_io.load(ii);
        ua = in_io.act[ii];
        g0 = in_io.hgen[ii];
        nst = in_io.nsteps[ii];
        d = in_io.draw[ii];
        pin(s); pin(ua); pin(g0); pin(nst); pin(d);
    }
    // the reset position (and its key) into LDS by Q3, which has no work in phase 0 (on Q0 the
    // wait for its load sat in front of ply 0's apply); read after ply 0's first barrier
    if (RR == 3 && l == 0) {
        const Pos rp = icd->pos;
        L.rp = rp;
        if (OCC) L.rkey0 = board_key(rp);
    }
    int a = (int)ua;
    DevHist h = DevHist{htab, in_io.hgen, g0, ii, HTAB_BITS};
    RepProbe pr;  // Q1: the window probe of the coming ply's pre-move board
    if (RR == 1 && live) rep_prefetch(h, s, pr);
    // Q1: the occupancy bitmap starts empty, so it mirrors a board's window only once that is
    // empty (from the launch's start, or at a reset / an irreversible move); until then the board
    // is probed in the table
    OccQ oq{RR == 1 && hl_of(s.meta) == 0, RR == 1, true, false};
    QuadPend pend{false, false, 0};  // Q0: the first ply's action is the env's
    const int wg_half = ((nn + QUAD_BOARDS * QUADS_WG - 1) / (QUAD_BOARDS * QUADS_WG)) >> 1;
#ifdef GC_PSTAMPS
    const unsigned long long g_pst_entry = pst_entry_where();
    unsigned long long rt1 = 0;
    if (l == 0) {
        for (int k = 0; k < 8; k++) gc_pst[threadIdx.x >> 6][k] = 0;
        gc_pst[threadIdx.x >> 6][8] = __builtin_amdgcn_s_memtime();
    }
    const unsigned long long rt0 = __builtin_amdgcn_s_memrealtime();
#endif
    // per-launch stats (ST), packed: a launch runs <= ROLLOUT_MAX_PLIES plies, so every count fits
    // 16 bits and the reward sum 32 -- four registers instead of nine
    u32 sa = 0, sb = 0, sc = 0;  // steps | errors << 16, mates | 3-folds << 16, move caps | no-moves << 16
    int32_t rsum = 0;
    StepOut o = {0, 0, R_NONE, 0};
    for (int p = 0; p < plies; p++) {
        // (GC_WG_FAIR, above: this workgroup's turn one level up)
#ifndef GC_TURN_SHIFT
#define GC_TURN_SHIFT 2  // turns of 4 plies: same box at K = 20, 8 repeats, 13.32 vs 13.01e9 (events
                         // 4.53 vs 4.66 us per ply; 8-ply turns 13.22); at K = 1 000 level (run_r06v, w)
#endif
        const bool up = GC_WG_FAIR && ((((int)blockIdx.x >= wg_half) ? 1 : 0) ^ ((p >> GC_TURN_SHIFT) & 1));
        o = quad_ply<RR, OCC>(L, C, l, i, live, s, a, d, h, nst, pr, pend, oq, up);
        const int played = a;  // (Q0: resolved at the ply's start; Q1: read after its barrier A)
#ifdef GC_PSTAMPS
        if (p == 0) rt1 = __builtin_amdgcn_s_memrealtime();
#endif
        if (RR == 1) {  // the ply's outputs (trace, stats) and the window write
            if (trace && live) trace[(size_t)p * nn + i] = trace_word(played == A_NONE ? -1 : played, o);
            if (!ST) {
            } else if (played == A_NONE) {
                sc += 1u << 16;
            } else {
                sa += 1u;
                rsum += o.reward;
                if (o.done) {
                    sb += (o.reason == R_MATE || o.reason == R_MATED ? 1u : 0u) | (o.reason == R_REPETITION ? 1u << 16 : 0u);
                    sc += (o.reason == R_MOVE_CAP ? 1u : 0u) | (o.reason == R_OPP_NO_MOVE ? 1u << 16 : 0u);
                    sa += o.reason == R_BOTH_CHECKED || o.reason == R_WINDOW_FULL ? 1u << 16 : 0u;
                }
            }
            h.commit();  // this ply's window write lands before the next ply's probe
        }
    }
#ifdef GC_PSTAMPS
    if (g_pst_out != nullptr && l == 0) {
        const size_t w = (size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
        for (int k = 0; k < 8; k++) g_pst_out[w * 12 + k] = gc_pst[threadIdx.x >> 6][k];
        g_pst_out[w * 12 + 8] = g_pst_entry;
        g_pst_out[w * 12 + 9] = rt0;
        g_pst_out[w * 12 + 10] = rt1;
        g_pst_out[w * 12 + 11] = __builtin_amdgcn_s_memrealtime();
    }
#endif
    if (!live || RR >= 2) return;
    const PairIO io = store_io(slab, nn);
    if (RR == 0) {
        a = pend.resolve(L, l, a);  // the next action (Q2's last pick arrived before the last barrier)
        io.act[i] = (uint16_t)a;
        io.draw[i] = d;
    } else {
        io.store(i, s);
        // (h.flush through io's freshly derived pointer: h's own, kept from the entry load across
        // the whole loop, was the kernel's one spill -- and a private segment slows every wave's launch)
        if (h.gen() != g0) io.hgen[i] = h.gen();
        io.nsteps[i] = nst;
        io.reward[i] = o.reward;
        io.done[i] = (uint8_t)o.done;
        io.reason[i] = (uint8_t)o.reason;
        if (ST) {
            uint64_t* so = stats + 8 * (size_t)i;
            so[0] += sa & 0xFFFFu; so[1] += (uint64_t)(int64_t)rsum;
            so[2 + R_MATE] += sb & 0xFFFFu; so[2 + R_REPETITION] += sb >> 16; so[2 + R_MOVE_CAP] += sc & 0xFFFFu;
            so[2 + R_NO_MOVES] += sc >> 16; so[2 + R_BOTH_CHECKED] += sa >> 16;
        }
    }
}

// The fused K-ply rollout on quads (k_env_rollout2's contract: same arguments, state, trace
// and stats).  Q0 writes the next action and draw counter, Q1 the rest, as W0 / W1 there.
template <bool OCC>
__global__ void __launch_bounds__(4 * QUAD_BOARDS * QUADS_WG) __attribute__((amdgpu_waves_per_eu(4)))
    k_env_rollout4(uint8_t* __restrict__ slab, int nn, uint64_t seed, u64* __restrict__ htab,
                   const uint16_t* __restrict__ racts, const EnvDev::InitCache* __restrict__ icd, u32 rinfo,
                   uint64_t* __restrict__ stats, u64* __restrict__ trace) {
    const int plies = (int)(rinfo >> 18);
    rinfo &= 0x1FFFFu;
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int qw = wv >> 2;  // the quad of this wave within the workgroup
#ifndef GC_QXOR
#define GC_QXOR 2  // the roles of a workgroup's second quad: SIMD s holds roles s and s ^ GC_QXOR
#endif
    const int role = (wv & 3) ^ ((qw & 1) ? GC_QXOR : 0);
    const int l = threadIdx.x & (QUAD_BOARDS - 1);
    const int i = (blockIdx.x * QUADS_WG + qw) * QUAD_BOARDS + l;
    // Issue priority: a SIMD hosts Q0 + Q2 or Q1 + Q3 (of both quads of a workgroup and of the
    // CU's other workgroup); the state-carrying roles hold the longer chains, so their waves
    // issue first (same-box A/B: 13.39-13.46 -> 14.21-14.25e9; Q1 alone 13.99-14.17).  Packed
    // 2-bit priority per role, GC_QPRIO for diagnostic builds.
#ifndef GC_QPRIO
#define GC_QPRIO 0x0A  // Q0 2, Q1 2, Q2 0, Q3 0
#endif
    switch ((GC_QPRIO >> (2 * role)) & 3) {  // (s_setprio takes an immediate)
        case 1: __builtin_amdgcn_s_setprio(1); break;
        case 2: __builtin_amdgcn_s_setprio(2); break;
        case 3: __builtin_amdgcn_s_setprio(3); break;
        default: break;
    }
    switch (role) {
        case 0: quad_run<0, false, OCC>(slab, nn, seed, htab, racts, icd, rinfo, plies, stats, trace, qw, l, i); break;
        case 1:
            if (stats) quad_run<1, true, OCC>(slab, nn, seed, htab, racts, icd, rinfo, plies, stats, trace, qw, l, i);
            else quad_run<1, false, OCC>(slab, nn, seed, htab, racts, icd, rinfo, plies, stats, trace, qw, l, i);
            break;
        case 2: quad_run<2, false, OCC>(slab, nn, seed, htab, racts, icd, rinfo, plies, stats, trace, qw, l, i); break;
        default: quad_run<3, false, OCC>(slab, nn, seed, htab, racts, icd, rinfo, plies, stats, trace, qw, l, i); break;
    }
    // The completion word: every workgroup, its stores performed (the barrier waits for them),
    // counts itself; the last one bumps the launch count and writes it to host-mapped memory,
    // where gc_env_wait_rollout sees it ~5 us before the stream's completion signal would tell
    // (the end-of-kernel write-back and the command processor's signal: tools/region_anatomy.hip).
    // A timing signal only -- the results are read through the stream, after the kernel's own
    // release -- so no fences: an agent-scope release per workgroup writes its XCD's L2 back
    // (+40 us per launch, measured).
    const EnvDev::InitCache::DoneWord dw = icd->done;
    if (dw.ctr) {
        __syncthreads();
        if (threadIdx.x == 0) {
            const u32 prev = __hip_atomic_fetch_add(dw.ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const u32 wgs = (u32)(nn + QUAD_BOARDS * QUADS_WG - 1) / (QUAD_BOARDS * QUADS_WG);  // (not gridDim: no implicit kernargs)
            if (prev == wgs - 1) {
                __hip_atomic_store(dw.ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const u32 v = __hip_atomic_fetch_add(dw.seq, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
                __hip_atomic_store(dw.host, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
}

// Fused K-ply random self-play: state in registers for the whole launch.  Per-ply outputs
// go to the optional trace [ply][N] (trace_word); the last ply's outputs and per-board stats
// [steps, reward_sum(two's complement), ends[0..5]] are written.
template <bool OPP>
__global__ void __launch_bounds__(BLOCK) k_env_rollout(EnvDev e, int plies, u64* trace, uint64_t* stats) {
    LDS_SCRATCH_DECL;
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= e.n) return;
    Pos s = e.st.load(i);
    u32 g0 = e.hgen[i], d = e.draw[i], ua = e.act[i];
    pin(s); pin(g0); pin(d); pin(ua);
    DevHist h = e.hist(i, g0);
    PolicyCtx pc = {e.seed, (u32)i, d};
    int a = (int)ua;
    uint64_t steps = 0, rsum = 0;
    u32 e_mate = 0, e_rep = 0, e_cap = 0, e_nomove = 0, e_err = 0;
    StepOut o = {0, 0, R_NONE, 0};
    for (int p = 0; p < plies; p++) {
        o = {0, 0, R_NONE, 0};
        Gen g;
        MoveSet ms;
        bool have = false;
        int played = a;
        if (a == A_NONE) {
            reset_board(e, s, h);
            o.reason = R_NO_MOVES;
            e_nomove++;
            played = -1;
        } else {
            o = OPP ? env_step_vs<false>(s, h, a, nullptr, g, ms, scr, pc) : env_step<false>(s, h, a, nullptr, g, ms, scr);
            have = o.moved;
            steps++;
            rsum += (uint64_t)(int64_t)o.reward;
            if (o.done) {
                e_mate += o.reason == R_MATE || o.reason == R_MATED;
                e_rep += o.reason == R_REPETITION;
                e_cap += o.reason == R_MOVE_CAP;
                e_err += o.reason == R_BOTH_CHECKED || o.reason == R_WINDOW_FULL;
                e_nomove += o.reason == R_OPP_NO_MOVE;
                reset_board(e, s, h);
                have = false;
            }
        }
        if (OPP && !have) after_reset<OPP>(e, s, h, g, ms, scr, pc);
        if (trace) trace[(size_t)p * e.n + i] = trace_word(played, o);
        a = selfplay_pick(s, pc);
        h.commit();
    }
    e.reward[i] = o.reward;  // the last ply's env.step() outputs (per-ply: trace buffers)
    e.done[i] = (uint8_t)o.done;
    e.reason[i] = (uint8_t)o.reason;
    e.st.store(i, s);
    h.flush(g0);
    e.draw[i] = pc.draw;
    e.act[i] = (uint16_t)a;
    e.nsteps[i] += (u32)steps;
    if (stats) {
        uint64_t* so = stats + 8 * (size_t)i;
        so[0] += steps; so[1] += rsum;
        so[2 + R_MATE] += e_mate; so[2 + R_REPETITION] += e_rep; so[2 + R_MOVE_CAP] += e_cap;
        so[2 + R_NO_MOVES] += e_nomove; so[2 + R_BOTH_CHECKED] += e_err;
    }
}

// ----------------------------------------------------------------------------- single-board env ops
// The primitive ops of one ChessEnvV2.step() for a host-side opponent policy (the
// single-board env gym_chess_amd.single.ChessEnv: the reference's opponents are host
// callables, "random" draws from numpy's global generator, chess_v2.py:116-127).  The env's
// bookkeeping (chess_v2.py:219-294) runs here on the device, split where the host policy
// must see the move list: AGENT = the agent's step up to the opponent's turn (validation,
// done / move-cap early returns, player_move incl. the 3-fold count of the pre-move board,
// the engine's both-kings-checked error, mate +100, and the move-count rule when no
// opponent follows), REPLY = the opponent's player_move (-its capture value, -100 if the
// agent is mated, the move-count rule), RESET = reset() up to the BLACK opening, OPEN = the
// opponent's opening move (3-fold verdict discarded, move_count 1), SYNC = no change.  Every
// op writes the resulting state, outputs and the side to move's move list in reference order
// into one host-mapped record (gc_single_record): one launch, no copy.
// SET = the state setter (chess_v2.py:315-323): the board and the six flags from the record's
// own fields (written by the host before the launch); the side to move, move_count, done and
// the 3-fold window stay, as in the reference.
enum { SOP_RESET = 0, SOP_AGENT = 1, SOP_REPLY = 2, SOP_OPEN = 3, SOP_SYNC = 4, SOP_SET = 5 };
static_assert(sizeof(gc_single_record) == 728, "gym_chess_amd.single._REC mirrors this layout");
// One op in three parts: single_begin (one lane: validation, the ply, the window) leaves the
// position in LDS; list_par (every lane) lists the side to move's moves -- their count decides
// a mate; single_end (one lane) settles the outcome, stores the state and fills the record.
struct SingleCtx {
    Pos s;
    Gen g;               // gen_init of s after a ply (shared with list_par)
    DevHist h;
    u32 g0;
    int status, reward, done, reason, chk, pend, white, flags, op, has_g;
    int cached;          // (the server) s and h.g hold the board's state and window generation
    unsigned long long t[3];  // (the server) begin / list / end done (s_memrealtime)
};
enum { SPEND_NONE = 0, SPEND_AGENT = 1, SPEND_REPLY = 2 };

// valid: the action's validity when the caller knows it (the server: membership in the list it
// made for this position), else -1 (action_legal on the position)
__device__ __noinline__ void single_begin(const EnvDev& e, int i, int op, int action, int flags, int valid,
                                          LdsScratch& scr, const gc_single_record* in, SingleCtx& c) {
    // the board's state: the server's copy from its last op, else from the env's memory
    Pos s = c.cached ? c.s : e.st.load(i);
    const u32 g0 = c.cached ? c.h.g : e.hgen[i];
    DevHist h = e.hist(i, g0);
    int status = 0, reward = 0, done = 0, reason = R_NONE, pend = SPEND_NONE;
    Gen g;
    MoveSet ms;
    int mr = 0;
    bool rep = false, chk = false;
    bool has_g = false;
    const bool white = (s.meta & M_WHITE) != 0;
    if (op == SOP_RESET) {  // chess_v2.py:183-206
        s = e.ic.pos;
        h.bump_gen();
    } else if (op == SOP_AGENT) {
        if (valid < 0) {
            Gen gs;
            gen_init(s, gs);
            valid = action_legal(s, gs, action) ? 1 : 0;
        }
        if (!valid) {  // 239-242: the state stays, done as it was
            reward = -10;
            done = (s.meta & M_DONE) ? 1 : 0;
            reason = R_INVALID;
        } else if (s.meta & M_DONE) {  // 245-251
            done = 1;
            reason = R_DONE_ALREADY;
        } else if (mc_of(s.meta) > MOVES_MAX) {  // 252-258
            done = 1;
            reason = R_MOVE_CAP;
        } else {
            const int rc = env_ply<0>(s, h, action, g, ms, scr, &mr, &rep, &chk);
            if (rc == 1) {
                status = 1;  // lib.rs:1442-1446: the engine raises, nothing changes
            } else {
                has_g = true;
                reward = -10 + mr;  // 261-264 (Q9)
                if (rep) { done = 1; reason = R_REPETITION; }
                if (rc == 2) { done = 1; reason = R_WINDOW_FULL; }
                pend = SPEND_AGENT;  // the mate test and the move-count rule wait for the list
            }
        }
    } else if (op == SOP_REPLY) {  // 275-292
        const int rc = env_ply<0>(s, h, action, g, ms, scr, &mr, &rep, &chk);
        if (rc == 1) {
            status = 1;
        } else {
            has_g = true;
            reward = -mr;
            if (rep) { done = 1; reason = R_REPETITION; }
            if (rc == 2) { done = 1; reason = R_WINDOW_FULL; }
            pend = SPEND_REPLY;
        }
    } else if (op == SOP_OPEN) {  // 208-216
        const int rc = env_ply<0>(s, h, action, g, ms, scr, &mr, &rep, &chk);
        if (rc == 1) status = 1;
        else { has_g = true; s.meta = (s.meta & ~(u32)M_DONE) + (1u << M_MC_SHIFT); }
    } else if (op == SOP_SET) {  // 315-323: board, rights, checks; nothing else changes
        const u32 m = (s.meta & ~(u32)(M_RIGHTS | M_WCHK | M_BCHK)) | (in->rights[0] ? M_WKC : 0u) |
                      (in->rights[1] ? M_WQC : 0u) | (in->rights[2] ? M_BKC : 0u) | (in->rights[3] ? M_BQC : 0u) |
                      (in->checked[0] ? M_WCHK : 0u) | (in->checked[1] ? M_BCHK : 0u);
        s = from_mailbox(in->board, m);
    }
    c.s = s; c.g = g; c.h = h; c.g0 = g0;
    c.status = status; c.reward = reward; c.done = done; c.reason = reason; c.chk = chk ? 1 : 0;
    c.pend = pend; c.white = white ? 1 : 0; c.flags = flags; c.op = op; c.has_g = has_g ? 1 : 0;
}

__device__ __noinline__ void single_end(const EnvDev& e, int i, int nmoves, SingleCtx& c, gc_single_record* __restrict__ rec) {
    Pos s = c.s;
    if (c.pend == SPEND_AGENT) {
        if (nmoves == 0 && c.chk) {  // 269-272
            s.meta |= M_DONE;
            c.done = 1;
            c.reward += 100;
            c.reason = R_MATE;
        }
        if (!c.done && !(c.flags & 1) && !c.white) s.meta += (1u << M_MC_SHIFT);  // 291-292, no opponent
    } else if (c.pend == SPEND_REPLY) {
        if (nmoves == 0 && c.chk) {
            s.meta |= M_DONE;
            c.done = 1;
            c.reward -= 100;
            c.reason = R_MATED;
        }
        if (s.meta & M_WHITE) s.meta += (1u << M_MC_SHIFT);
    }
    if (c.status == 0 && c.op != SOP_SYNC) {
        c.h.commit();
        e.st.store(i, s);
        c.h.flush(c.g0);
    }
    c.s = s;  // (the server keeps it for its next op)
    rec->status = c.status;
    rec->reward = c.reward;
    rec->done = (uint8_t)c.done;
    rec->reason = (uint8_t)c.reason;
    rec->env_done = (s.meta & M_DONE) ? 1 : 0;
    rec->white_to_move = (s.meta & M_WHITE) ? 1 : 0;
    rec->rights[0] = (s.meta & M_WKC) != 0; rec->rights[1] = (s.meta & M_WQC) != 0;
    rec->rights[2] = (s.meta & M_BKC) != 0; rec->rights[3] = (s.meta & M_BQC) != 0;
    rec->checked[0] = (s.meta & M_WCHK) != 0; rec->checked[1] = (s.meta & M_BCHK) != 0;
    rec->move_count = (uint16_t)mc_of(s.meta);  // (the board: every lane, single_run)
}

// the three parts of one op on a 64-lane workgroup (c, lrec in LDS); valid as single_begin's
__device__ __forceinline__ void single_run(const EnvDev& e, int i, int op, int action, int flags, int valid,
                                           LdsScratch& scr, const gc_single_record* in, SingleCtx& c,
                                           gc_single_record& lrec) {
    if (threadIdx.x == 0) {
        single_begin(e, i, op, action, flags, valid, scr, in, c);
        c.t[0] = __builtin_amdgcn_s_memrealtime();
    }
    __syncthreads();
    list_par(c.s, GC_SINGLE_MOVES_CAP, lrec.moves, &lrec.nmoves, c.has_g ? &c.g : nullptr);  // every lane
    __syncthreads();
    if (threadIdx.x == 0) {
        c.t[1] = __builtin_amdgcn_s_memrealtime();
        single_end(e, i, lrec.nmoves, c, &lrec);
        c.t[2] = __builtin_amdgcn_s_memrealtime();
    }
    __syncthreads();
    lrec.board[threadIdx.x & 63] = (int8_t)id_at(c.s, (int)(threadIdx.x & 63));  // the mailbox, a square per lane
    __syncthreads();
}

// copy the record (LDS) to the host-mapped one, every lane
__device__ __forceinline__ void single_publish(const gc_single_record& lrec, gc_single_record* __restrict__ hrec) {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(&lrec);
    uint32_t* dst = reinterpret_cast<uint32_t*>(hrec);
    const int words = (int)(offsetof(gc_single_record, moves) / 4) + (lrec.nmoves < GC_SINGLE_MOVES_CAP ? lrec.nmoves : GC_SINGLE_MOVES_CAP + 1) / 2 + 1;
    for (int k = threadIdx.x; k < words && k < (int)(sizeof(gc_single_record) / 4); k += 64) dst[k] = src[k];
    __threadfence_system();  // the record lives in host memory
}

__global__ void __launch_bounds__(64) k_single(EnvDev e, int i, int op, int action, int flags,
                                               gc_single_record* __restrict__ hrec) {
    __shared__ u64 lds_scr[SCRATCH_SLOTS * BLOCK];
    __shared__ gc_single_record lrec;  // built here, then written to host memory by every lane
    __shared__ __attribute__((aligned(16))) unsigned char c_raw[sizeof(SingleCtx)];  // (SingleCtx has default member initialisers)
    SingleCtx& c = *reinterpret_cast<SingleCtx*>(c_raw);
    LdsScratch scr{lds_scr + threadIdx.x};
    if (threadIdx.x == 0) c.cached = 0;
    single_run(e, i, op, action, flags, -1, scr, hrec, c, lrec);
    single_publish(lrec, hrec);
}

// ----------------------------------------------------------------------------- single-board server
// The single-board env's ops without a launch each (one step paid a
// ~25 us launch round trip -- tools/region_anatomy.hip -- plus k_single's cold loads): one
// wave stays resident on its own stream and serves requests through a host-mapped mailbox.
// The host writes the request, then bumps req_seq; the wave polls req_seq (system-scope loads,
// s_sleep between), runs the same single_run, writes the record to host memory and then
// resp_seq.  It exits on QUIT, or when no request came for SRV_IDLE_MS (so it has always
// drained before its process can end); the host starts it again on the next request.
struct SrvBox {
    // the request: one 16-byte read on the device (the host writes op / action / flags, then seq)
    u32 req_seq, op;
    int32_t action;
    u32 flags;
    u32 pad1[12];
    u32 resp_seq, pad2[15];  // own cache line
    u32 exited, pad3[15];    // the launch id of the last server that exited
    // the last op's segments (10 ns ticks): request read + validation, begin, list, end, record copy, idle wait
    u32 stamps[6];
};
#define SRV_QUIT 99
#define SRV_IDLE_MS 50
__device__ __forceinline__ u32 srv_load(const u32* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); }
__device__ __forceinline__ void srv_store(u32* p, u32 v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); }
__global__ void __launch_bounds__(64) k_single_server(EnvDev e, int i, SrvBox* box, gc_single_record* __restrict__ hrec,
                                                      u32 done_seq, u32 launch_id) {
    __shared__ u64 lds_scr[SCRATCH_SLOTS * BLOCK];
    __shared__ gc_single_record lrec;  // the last op's record: its move list validates the next AGENT
    __shared__ __attribute__((aligned(16))) unsigned char c_raw[sizeof(SingleCtx)];  // (SingleCtx has default member initialisers)
    SingleCtx& c = *reinterpret_cast<SingleCtx*>(c_raw);
    LdsScratch scr{lds_scr + threadIdx.x};
    if (threadIdx.x == 0) c.cached = 0;
    single_run(e, i, SOP_SYNC, 0, 0, 0, scr, hrec, c, lrec);  // the current position's list
    if (threadIdx.x == 0) c.cached = 1;  // from here on the board's state lives here (and is stored after every op)
    unsigned long long idle0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
    for (;;) {
        // the request in one 16-byte read from host memory: {seq, op, action, flags} (the host
        // writes seq last, so a new seq comes with its fields)
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 rq = *reinterpret_cast<const volatile u32x4*>(box);
        const u32 req = __builtin_amdgcn_readfirstlane(rq.x);
        if (req == done_seq) {
            if (__builtin_amdgcn_s_memrealtime() - idle0 > (unsigned long long)SRV_IDLE_MS * 100000ull) break;
            __builtin_amdgcn_s_sleep(8);
            continue;
        }
        const unsigned long long t_seen = __builtin_amdgcn_s_memrealtime();
        __atomic_thread_fence(__ATOMIC_ACQUIRE);  // SET's inputs (the record) after req_seq
        const int op = (int)__builtin_amdgcn_readfirstlane(rq.y);
        if (op == SRV_QUIT) break;
        const int action = (int)__builtin_amdgcn_readfirstlane(rq.z);
        const int flags = (int)__builtin_amdgcn_readfirstlane(rq.w);
        // chess_v2.py:240: the action against the list this server made for the position
        bool hit = false;
        for (int k = (int)threadIdx.x; k < lrec.nmoves && k < GC_SINGLE_MOVES_CAP; k += 64) hit |= lrec.moves[k] == (uint16_t)action;
        const int valid = __ballot(hit) != 0 ? 1 : 0;
        __syncthreads();
        const unsigned long long t_op = __builtin_amdgcn_s_memrealtime();
        single_run(e, i, op, action, flags, valid, scr, hrec, c, lrec);
        const unsigned long long t_list = __builtin_amdgcn_s_memrealtime();
        single_publish(lrec, hrec);  // the record, then the response
        __syncthreads();
        if (threadIdx.x == 0) {
            const unsigned long long t_copy = __builtin_amdgcn_s_memrealtime();
            srv_store(&box->stamps[0], (u32)(t_op - t_seen));
            srv_store(&box->stamps[1], (u32)(c.t[0] - t_op));
            srv_store(&box->stamps[2], (u32)(c.t[1] - c.t[0]));
            srv_store(&box->stamps[3], (u32)(c.t[2] - c.t[1]));
            srv_store(&box->stamps[4], (u32)(t_copy - t_list));
            srv_store(&box->stamps[5], (u32)(t_seen - idle0));
            srv_store(&box->resp_seq, req);
        }
        done_seq = req;
        idle0 = __builtin_amdgcn_s_memrealtime();
    }
    __threadfence_system();  // every op's state stores, then the exit mark
    if (threadIdx.x == 0) srv_store(&box->exited, launch_id);
}

// ----------------------------------------------------------------------------- engine server
// The drop-in ChessEngine's one-position calls (n = 1, reference rules) without a launch each:
// the single-board server's scheme (one resident wave, a host-mapped mailbox, s_sleep polling,
// idle exit) over stateless ops -- the request carries the state dict's board and flags, the
// response the list / castle word / next state.  Same device functions as the batched kernels
// (list_par = list_one with the lanes, next_state_one, check_flags).
enum { ENG_LIST = 1, ENG_CASTLE = 2, ENG_NEXT = 3, ENG_UPDATE = 4 };
#define ENG_SRV_CAP 320
struct EngBox {
    u32 req_seq, op, white, arg;  // arg: attack (LIST) or the action (NEXT); the host writes req_seq last
    u32 pad0[12];
    int8_t board[64];             // the request's state (mailbox + the import's meta bytes)
    uint8_t meta[8];
    u32 pad1[14];
    u32 resp_seq, count;          // count: the list's length, or the castle word
    int32_t reward, status;
    u32 pad2[12];
    int8_t out_board[64];
    uint8_t out_meta[8];
    u32 pad3[14];
    uint16_t moves[ENG_SRV_CAP];
    u32 exited, pad4[15];
};
__global__ void __launch_bounds__(64) k_engine_server(EngBox* box, u32 done_seq, u32 launch_id) {
    __shared__ __attribute__((aligned(16))) int8_t in[80];  // board 64 + meta 8 (+ pad)
    __shared__ __attribute__((aligned(16))) int8_t ob[64];
    __shared__ uint8_t om[8];
    __shared__ uint16_t mv[ENG_SRV_CAP];
    __shared__ int32_t cnt, rw, st;
    __shared__ Pos tp;  // NEXT / UPDATE: the new state, for the lanes' mailbox squares
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const int lane = (int)threadIdx.x;
    unsigned long long idle0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        const u32x4 rq = *reinterpret_cast<const volatile u32x4*>(box);
        const u32 req = __builtin_amdgcn_readfirstlane(rq.x);
        if (req == done_seq) {
            if (__builtin_amdgcn_s_memrealtime() - idle0 > (unsigned long long)SRV_IDLE_MS * 100000ull) break;
            __builtin_amdgcn_s_sleep(8);
            continue;
        }
        __atomic_thread_fence(__ATOMIC_ACQUIRE);  // the state after req_seq
        const int op = (int)__builtin_amdgcn_readfirstlane(rq.y);
        if (op == SRV_QUIT) break;
        const bool white = __builtin_amdgcn_readfirstlane(rq.z) != 0;
        const int arg = (int)__builtin_amdgcn_readfirstlane(rq.w);
        if (lane < 5)  // the 72 request bytes in five 16-byte reads
            reinterpret_cast<u32x4*>(in)[lane] = reinterpret_cast<const volatile u32x4*>(box->board)[lane];
        __syncthreads();
        const uint8_t side = white ? 1 : 0;
        // LIST / CASTLE: the player argument is the side to generate for (lib.rs:1454-1499);
        // NEXT / UPDATE keep the state's own current_player
        const Pos s = import_one(in, reinterpret_cast<const uint8_t*>(in + 64),
                                 (op == ENG_LIST || op == ENG_CASTLE) ? &side : nullptr, 0);
        int nout = 0;  // result u32 words to copy
        if (op == ENG_LIST) {
            list_par(s, ENG_SRV_CAP, mv, &cnt, nullptr, arg != 0);
            __syncthreads();
            nout = (cnt < ENG_SRV_CAP ? cnt : ENG_SRV_CAP) + 1;
            nout /= 2;
        } else if (op == ENG_CASTLE) {
            if (lane == 0) {
                Gen g;
                gen_init(s, g);
                int c = 0;
                if (g.castles & 1) c |= g.white ? (1 << 1) : (1 << 3);
                if (g.castles & 2) c |= g.white ? (1 << 0) : (1 << 2);
                cnt = c;
            }
        } else {  // NEXT / UPDATE: the move and flags on lane 0, the mailbox a square per lane
            if (lane == 0) {
                Pos t = s;
                if (op == ENG_NEXT) {
                    const uint16_t a = (uint16_t)arg;
                    t = next_state_one(s, &side, &a, &rw, &st, 0);
                } else {
                    t.meta = (t.meta & ~(u32)(M_WCHK | M_BCHK)) | check_flags(t);
                    rw = 0;
                    st = 0;
                }
                export_one(t, nullptr, om, 0);
                tp = t;
            }
            __syncthreads();
            ob[lane] = (int8_t)id_at(tp, lane);
        }
        __syncthreads();
        // the response: results, a system-scope fence, then resp_seq
        if (op == ENG_LIST) {
            for (int k = lane; k < nout; k += 64) reinterpret_cast<u32*>(box->moves)[k] = reinterpret_cast<const u32*>(mv)[k];
        } else if (op == ENG_NEXT || op == ENG_UPDATE) {
            if (lane < 16) reinterpret_cast<u32*>(box->out_board)[lane] = reinterpret_cast<const u32*>(ob)[lane];
            else if (lane < 18) reinterpret_cast<u32*>(box->out_meta)[lane - 16] = reinterpret_cast<const u32*>(om)[lane - 16];
            if (lane == 0) {
                box->reward = rw;
                box->status = st;
            }
        }
        if (lane == 0) box->count = (u32)cnt;
        __threadfence_system();
        __syncthreads();
        if (lane == 0) srv_store(&box->resp_seq, req);
        done_seq = req;
        idle0 = __builtin_amdgcn_s_memrealtime();
    }
    __threadfence_system();
    if (lane == 0) srv_store(&box->exited, launch_id);
}

// the live 3-fold window of board i (its table entries, then its spill entries): boards and
// occurrence counts (diagnostic readout; ChessEnv.saved_boards)
__global__ void k_window_boards(EnvDev e, int i, int8_t* __restrict__ boards, uint8_t* __restrict__ counts, int cap,
                                int* __restrict__ n) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const u32 g = e.hgen[i];
    DevHist h = e.hist(i, g);
    int k = 0;
    for (int pos = 0; pos < (1 << h.bits()); pos++) {
        const RepEntry x = h.load(pos);
        if ((u32)x.hdr != g) continue;
        if (k < cap) {
            to_mailbox(Pos{x.k, x.q, x.r, x.b, x.n, x.p, x.w, 0}, boards + 64 * (size_t)k);
            counts[k] = (uint8_t)(x.hdr >> 56);
        }
        k++;
    }
    const SpillTab& sp = h.sp;
    for (u32 t = 0; sp.ent && t <= sp.mask; t++) {
        const u64* x = sp.ent + (size_t)t * 8;
        if (sp_owner1(x[0]) != (u32)i + 1 || sp_gen(x[0]) != g) continue;
        if (k < cap) {
            to_mailbox(Pos{x[1], x[2], x[3], x[4], x[5], x[6], x[7], 0}, boards + 64 * (size_t)k);
            counts[k] = (uint8_t)sp_cnt(x[0]);
        }
        k++;
    }
    *n = k;
}

// Column sums of the per-board rollout stats [n][8] into out[8] (zeroed by the caller): a
// wave-level butterfly per column, one atomic per column per wave.  Copying the 64 B/board
// table to the host and summing there cost more than the rollout itself at 65 536 boards.
__global__ void __launch_bounds__(BLOCK) k_sum_stats(const uint64_t* __restrict__ stats, int n,
                                                     unsigned long long* __restrict__ out) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        unsigned long long v = i < n ? stats[8 * (size_t)i + k] : 0ull;
#pragma unroll
        for (int off = 32; off; off >>= 1) v += __shfl_xor(v, off, 64);
        if ((threadIdx.x & 63) == 0 && v) atomicAdd(out + k, v);
    }
}

// ----------------------------------------------------------------------------- API step
// The reference's step() call shape for a policy that lives on the GPU: an external action
// per board in, and out everything ChessEnvV2.step() hands back (chess_v2.py:219-294) plus
// the rebuilt possible_actions (333-335) -- reward, done, info reason, the observation
// (int8 mailbox, 153-158), the legal-action mask and count -- written straight into the
// caller's device buffers.  Optional: auto-reset of finished boards (a vector-env
// convention; the reference resets on the caller's reset()) and the random policy's pick
// over the new list (a ready-made next action; also becomes the env's act[]).

// legal-action mask of the position gen_moves described, WORD-MAJOR: o[f * n] = targets of
// from-square f of this board (o = mask + board), o[64 * n] bit c = action 4096 + c (castles).
// Word-major so that each of the 65 stores of a wave writes 512 contiguous bytes: every word
// is first zeroed (coalesced), then the own pieces' words are written (at most 16 of them;
// the parked slot of the j-th own piece is slot j, fast pawns from their origin sets).
template <class S>
__device__ void write_mask(const Pos& s, const Gen& g, const MoveSet& ms, const S& scr, u64* __restrict__ o,
                           size_t n) {
    u64 c = 0;
    if (g.castles & 1) c |= g.white ? (1ull << 1) : (1ull << 3);  // QS: 4097 / 4099
    if (g.castles & 2) c |= g.white ? (1ull << 0) : (1ull << 2);  // KS: 4096 / 4098
#pragma unroll 8
    for (int sq = 0; sq < 64; sq++) o[sq * n] = 0;
    o[64 * n] = c;
    u64 pcs = g.own;
    for (int j = 0; pcs; j++) {
        int sq = ctz(pcs);
        pcs &= pcs - 1;
        u64 w = ms.big ? legal_targets(s, g, sq, type_at(s, sq))
                       : (((ms.fastp >> sq) & 1) ? fast_pawn_targets(ms, sq, g.white) : scr.get(j));
        if (w) o[sq * n] = w;
    }
}

// spread the 8 bits of b over the 8 bytes of a word (bit j -> byte j, value 0/1): byte j
// keeps bit j of a broadcast copy, then "nonzero -> 1" per byte (no carries: bytes <= 255)
__device__ __forceinline__ u64 bits_to_bytes(u32 b) {
    u64 y = ((u64)(b & 0xFFu) * 0x0101010101010101ull) & 0x8040201008040201ull;
    return ((y + 0x7F7F7F7F7F7F7F7Full) >> 7) & 0x0101010101010101ull;
}
// 4 bits of b -> the 4 bytes of a word (bit j -> byte j, value 0/1), in 32-bit arithmetic
__device__ __forceinline__ u32 nib_to_bytes(u32 b) {
    const u32 y = ((b & 0xFu) * 0x01010101u) & 0x08040201u;
    return ((y + 0x7F7F7F7Fu) >> 7) & 0x01010101u;
}
// int8 mailbox of the position (lib.rs:41-50 ids), 16 words of 4 squares: the id's three bits
// as three planes (K 1, Q 2, R 3, B 4, N 5, P 6), each spread to bytes and weighted, black
// bytes negated in two's complement (no byte overflows: every byte <= 6)
__device__ __forceinline__ u32 obs_word(u64 b0, u64 b1, u64 b2, u64 blk, int sh) {
    const u32 v = nib_to_bytes((u32)(b0 >> sh)) + (nib_to_bytes((u32)(b1 >> sh)) << 1) +
                  (nib_to_bytes((u32)(b2 >> sh)) << 2);
    const u32 b = nib_to_bytes((u32)(blk >> sh));
    return (v ^ (b * 0xFFu)) + b;
}
__device__ void write_obs(const Pos& s, int8_t* __restrict__ out) {
    u64* o = reinterpret_cast<u64*>(out);
    const u64 b0 = s.k | s.r | s.n, b1 = s.q | s.r | s.p, b2 = s.b | s.n | s.p;
    const u64 blk = occ_of(s) & ~s.w;
#pragma unroll
    for (int r = 0; r < 8; r++)
        o[r] = (u64)obs_word(b0, b1, b2, blk, 8 * r) | ((u64)obs_word(b0, b1, b2, blk, 8 * r + 4) << 32);
}

#define WRITE_OBS_Q3(fs, base, i, nn) write_obs(fs, (base) + 64 * (size_t)(i))


template <bool OPP>
__global__ void __launch_bounds__(BLOCK) k_env_step_api(EnvDev e, const uint16_t* __restrict__ acts,
                                                        int32_t* __restrict__ rw, uint8_t* __restrict__ dn,
                                                        uint8_t* __restrict__ rs, u64* __restrict__ mask,
                                                        int8_t* __restrict__ obs, int32_t* __restrict__ cnt,
                                                        uint16_t* __restrict__ pick_out, int autoreset, size_t mstride) {
    LDS_SCRATCH_DECL;
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= e.n) return;
    Pos s = e.st.load(i);
    u32 g0 = e.hgen[i], d = e.draw[i], nst = e.nsteps[i];
    int a = (int)acts[i];
    pin(s); pin(g0); pin(d); pin(nst);
    DevHist h = e.hist(i, g0);
    PolicyCtx pc = {e.seed, (u32)i, d};
    Gen gv, g;
    MoveSet ms;
    gen_init(s, gv);
    StepOut o = OPP ? env_step_vs<true>(s, h, a, &gv, g, ms, scr, pc) : env_step<true>(s, h, a, &gv, g, ms, scr);
    bool have = o.moved;
    nst += 1;
    if (autoreset && o.done) {
        reset_board(e, s, h);
        after_reset<OPP>(e, s, h, g, ms, scr, pc);
        have = true;
    }
    if (!have) {  // state unchanged (invalid action, done, move cap, both kings checked)
        gen_init(s, g);
        gen_moves(s, g, ms, scr);
    }
    rw[i] = o.reward;
    dn[i] = (uint8_t)o.done;
    rs[i] = (uint8_t)o.reason;
    if (cnt) cnt[i] = ms.total;
    if (mask) write_mask(s, g, ms, scr, mask + i, mstride);
    if (obs) write_obs(s, obs + 64 * (size_t)i);
    if (pick_out) {
        uint16_t p = pick_mask_order(s, g, ms, scr, e.seed, i, pc.draw);
        pick_out[i] = p;
        e.act[i] = p;
    }
    h.commit();
    e.st.store(i, s);
    h.flush(g0);
    e.draw[i] = pc.draw;
    e.nsteps[i] = nst;
    e.reward[i] = o.reward;
    e.done[i] = (uint8_t)o.done;
    e.reason[i] = (uint8_t)o.reason;
}

// ----------------------------------------------------------------------------- API step, paired
// k_env_step_api (opponent "none") on the paired driver.  W0 validates the external action
// on the pre-move board (quick_legal: a king move's target is attack-tested alone, no enemy
// map; chess_v2.py:240) and applies it; one pair_half generates the next side's moves, or --
// for a board whose state stays (invalid action, done, move cap) -- its own moves again
// (regen).  Phase 3: both waves settle the outcome (env_step<VALIDATE = true>); W0 completes
// the parked targets (fast pawns, or a reset board's cached set) and picks; each wave writes
// half of the square-major mask; W1 the observation and outputs.  A board left with both
// kings checked and no reset (weird positions only) regenerates alone, without slots.
struct ApiOut {
    int32_t* rw;
    uint8_t* dn;
    uint8_t* rs;
    u64* mask;
    int8_t* obs;
    int32_t* cnt;
    uint16_t* pick;
    size_t ms;  // the mask's row stride in words (gc_env_step_device2; default n)
};
__device__ __forceinline__ void ic_moves(const EnvDev::InitCache& ic, Gen& g, MoveSet& ms) {
    g.white = ic.white;
    g.own = ic.own;
    g.castles = ic.castles;
    ms.fastp = ic.fastp; ms.o1 = ic.o1; ms.o2 = ic.o2; ms.ol = ic.ol; ms.orr = ic.orr;
#pragma unroll
    for (int b = 0; b < 5; b++) ms.cnt[b] = ic.cnt[b];
    ms.total = ic.total;
    ms.big = false;
}

// ----------------------------------------------------------------------------- API step, quads
// The API step (external actions in; reward / done / reason, the observation, the legal-action
// mask and count, the random policy's pick out; auto-reset) on FOUR waves per 64 boards, as the
// headline rollout's quads (k_env_rollout4).  16 argument dwords, no padding (all preloaded): the
// output pointers live in device memory (outp, rewritten only when the caller's buffers change),
// auto-reset rides in rinfo bit 17.  The round-2 paired API step (k_env_step_api2, removed in
// round 6) ran each board's step as two long dependency chains on two waves and wrote its 34 MB
// legal-action mask at the end, when every workgroup finished at once.
//
//   phase 0   Q0: applies the action (speculatively: it is validated beside it)
//             Q1: the window probe of the pre-move board, the Philox word, the reset-table pick
//             Q2, Q3: validate the action (chess_v2.py:240-242), quick_legal in two halves:
//                 Q3 the move's shape (quick_pseudo), Q2 the king's safety (quick_safe)
//   phase 1   Q0: checkers, check mask, pins                  Q1: the mover's own check flag
//             Q2: enemy leaper + orthogonal slider attacks    Q3: enemy diagonal slider attacks
//   phase 2   Q0: castles, pawns (set-wise; every pawn's targets parked too)
//             Q1: knights, kings, then the 3-fold commit (its probe lands meanwhile)
//             Q2: queens                                      Q3: rooks, bishops
//             (pieces parked per ordinal in LDS with bit-sliced counts, as gen_moves)
//   phase 3   every role: the step's outcome (identical arithmetic on the same LDS data) and
//             its 16 mask rows, each written once, whole (a reset board: the start position's
//             rows, from the init cache); Q2: the pick (action-id order), the count, the env's
//             next action; Q3: the observation; Q1: the outputs, the state and the window.
// A mask row is written only by the role that owns its square.  (Zeroing the unoccupied
// squares' rows in phase 1 instead wrote partial rows twice: 28.4 vs 18.5 us per launch,
// measured in round 5.)  Boards outside
// the fast path -- > 16 own pieces, or both kings checked after the move (the move is void and
// the pre-move board regenerates) -- take the per-piece fallback (legal_targets) in phase 3,
// each role for its own rows.  Quad roles run only with the start position's pick table, as
// the rollout's.
struct ApiQuadLds {
    u64 slots[SCRATCH_SLOTS][QUAD_BOARDS];  // parked targets per own-piece ordinal (Q0, Q2, Q3)
    u64 ns[NBB][QUAD_BOARDS];               // Q0 -> all: the post-move board (if the action is valid)
    u32 nmeta[QUAD_BOARDS];
    int32_t mr[QUAD_BOARDS];                //           its capture reward
    u32 irrev[QUAD_BOARDS];                 //           irreversible move
    u32 valid[2][QUAD_BOARDS];              // Q3 ([0]: its shape), Q2 ([1]: king safety) -> all
    u64 pin3[3][QUAD_BOARDS];               // Q0 -> Q2, Q3: check mask, pinned, pin rays
    u32 f0[QUAD_BOARDS];                    // Q0 -> all: the side to move is in check
    u64 enemy[3][QUAD_BOARDS];              // Q2 ([1]), Q3 ([2]) -> Q0, Q2, Q3: the enemy map's parts
    u32 f1[QUAD_BOARDS];                    // Q1 -> all: the mover is in check after its move
    u64 cbw[4][2][QUAD_BOARDS];             // per role -> Q2: its pieces' move counts, a byte per ordinal
    u32 part[4][QUAD_BOARDS];               // move totals (Q0's holds the castles; Q3's a big board's)
    u32 castles[QUAD_BOARDS];               // Q0 -> all
    u32 rep[QUAD_BOARDS];                   // Q1 -> all: 3-fold count | window length << 8
    u32 x0[QUAD_BOARDS];                    // Q1 -> Q2: the Philox word of the draw
    u32 ra[QUAD_BOARDS];                    // Q1 -> Q2: the start-position table pick
};
__shared__ ApiQuadLds g_apiq_lds[QUADS_WG];
// phase 2's pieces: Q0 pawns | Q1 knights, kings | Q2 queens | Q3 rooks, bishops (same-box 17.13 us
// per launch; bishops on Q2 17.34; and the knights on Q0 17.60)
__device__ __forceinline__ void apiq_store(u64* p, u64 v) {
    __builtin_nontemporal_store(v, p);  // the mask rows stream (3.105-3.121 vs 3.049-3.104e9, round 4)
}

// Parked targets by own-piece ordinal in LDS (slot j of lane l at base[j * 64]), and each piece's
// move count as byte j of two words: the pick in action-id order (ascending from-square, the
// ordinals' order, then target) finds the piece by byte prefix sums instead of the bit-sliced
// per-square count planes (5 more 64-bit updates per piece, kPlanes)
struct OrdScratch {
    static constexpr bool kPark = true;
    static constexpr bool kPlanes = false;
    u64* base;
    u64 c0, c1;
    __device__ void put(int j, u64 v) {
        base[j * QUAD_BOARDS] = v;
        const u64 add = (u64)popc(v) << (8 * (j & 7));
        c0 |= j < 8 ? add : 0ull;
        c1 |= j < 8 ? 0ull : add;
    }
    __device__ u64 get(int j) const { return base[j * QUAD_BOARDS]; }
};
// the k-th (< normal) non-castle move in action-id order from the ordinal byte counts
__device__ __forceinline__ int ord_pick(const OrdScratch& scr, u64 own, u64 c0, u64 c1, int normal, int k) {
    int j;
    if (normal < 256) {
        const u64 cw[4] = {c0, c1, 0ull, 0ull};
        j = sw_locate(cw, k);
    } else {  // (never in play: byte prefix sums would overflow)
#pragma unroll 1
        for (j = 0; j < SCRATCH_SLOTS - 1; j++) {
            const int c = (int)(((j < 8 ? c0 : c1) >> (8 * (j & 7))) & 0xFF);
            if (k < c) break;
            k -= c;
        }
    }
    const int sq = kth_set_bit(own, j);
    return sq * 64 + kth_set_bit(scr.get(j), k);
}

// The per-piece fallback of one board (apiq_run: both kings checked, or > 16 own pieces), each
// part with its own context (gen_init) in its own scope
template <int R>
__device__ __noinline__ void apiq_slow_rows(Pos b, u64* __restrict__ o, size_t N) {  // (by value: no stack)
    Gen g;
    gen_init(b, g);
    for (int k = 0; k < 16; k++) {
        const int sq = 16 * R + k;
        const u64 w = ((g.own >> sq) & 1) ? legal_targets(b, g, sq, type_at(b, sq)) : 0ull;
        apiq_store(o + sq * N, w);
    }
}
__device__ __noinline__ u32 apiq_slow_castles(Pos b) {
    Gen g;
    gen_init(b, g);
    return g.castles;
}
// -> the legal count << 16 | the pick (A_NONE without a move)
__device__ __noinline__ u32 apiq_slow_pick(Pos b, u32 x0) {
    Gen g;
    gen_init(b, g);
    const int tot = count_legal(b, g);
    if (tot == 0) return (u32)A_NONE;
    MoveSet ms;
    moveset_clear(ms);
    ms.big = true;  // (select_action's per-piece path: no parked targets read)
    ms.total = tot;
    return ((u32)tot << 16) | (u32)select_action(b, g, ms, NoScratch{}, (int)scale_rank(x0, (u32)tot));
}

template <int RR>
__device__ __forceinline__ void apiq_run(uint8_t* __restrict__ slab, uint64_t seed, u64* __restrict__ htab,
                                         const uint16_t* __restrict__ racts, const EnvDev::InitCache* __restrict__ icd,
                                         const uint16_t* __restrict__ acts, const ApiOut& out, int nn, u32 rinfo,
                                         int qw, int l, int i) {
    ApiQuadLds& L = g_apiq_lds[qw];
    const int autoreset = (rinfo >> 17) & 1;
    rinfo &= 0x1FFFFu;
    const bool live = i < nn;
    const int ii = live ? i : nn - 1;  // dead lanes read a valid board, store nothing
    const size_t N = out.ms;  // the mask rows' stride
    const PairIO in_io(slab, nn);
    const PairCtx C = {seed, htab, in_io.hgen, racts, icd, (rinfo >> 16) != 0, rinfo & 0xFFFFu};
    // every role reads the pre-move board and the action (the stateless roles decide the outcome
    // and the fallback boards themselves); Q1 / Q2 the draw counter, Q1 the window and step counter
#ifdef GC_PSTAMPS
    const unsigned long long pst_entry = __builtin_amdgcn_s_memrealtime();
    if (l == 0) {
        for (int k = 0; k < 8; k++) gc_pst[threadIdx.x >> 6][k] = 0;
        gc_pst[threadIdx.x >> 6][8] = __builtin_amdgcn_s_memtime();
    }
#endif
    Pos s = in_io.load(ii);
    u32 ua = acts[ii], g0 = 0, nst = 0, d = 0;
    if (RR == 1) { g0 = in_io.hgen[ii]; nst = in_io.nsteps[ii]; }
    if (RR == 1 || RR == 2) d = in_io.draw[ii];
    pin(s); pin(ua); pin(g0); pin(nst); pin(d);
    PST(7);  // (GC_PSTAMPS: segment 7 = the entry loads; 0-6 phase 0, wait A, ..., phase 3)
#ifdef GC_PSTAMPS
    const unsigned long long pst_rt0 = __builtin_amdgcn_s_memrealtime();
#endif
    const int a = (int)ua;
    DevHist h = DevHist{htab, in_io.hgen, g0, ii, HTAB_BITS};
    OrdScratch scr{&L.slots[0][l], 0ull, 0ull};
    // issue priority: the state-carrying roles' chains are the longer; Q2 (a validation half,
    // on Q0's SIMDs) level with Q0 in phase 0
    // (Q3 raised as well, in phases 0 and 3: not faster)
    if (RR != 3) __builtin_amdgcn_s_setprio(2);
    const bool done0 = (s.meta & M_DONE) != 0;   // chess_v2.py:245-251
    const bool cap = mc_of(s.meta) > MOVES_MAX;  // 252-258
    const bool white = (s.meta & M_WHITE) != 0;
    const bool pre = live && !done0 && !cap;

    // ---- phase 0
    RepProbe pr;
    uint16_t ra = (uint16_t)A_NONE;
    if (RR == 0) {  // applied whatever the verdict: a board whose action is invalid keeps s
        Pos ns = s;
        ns.meta = (ns.meta & ~(u32)M_RIGHTS) | eff_rights(s);  // State::new
        int mr = 0;
        bool irrev = false;
        apply_legal(ns, white, a, &mr, &irrev);
        L.ns[0][l] = ns.k; L.ns[1][l] = ns.q; L.ns[2][l] = ns.r; L.ns[3][l] = ns.b;
        L.ns[4][l] = ns.n; L.ns[5][l] = ns.p; L.ns[6][l] = ns.w;
        L.nmeta[l] = ns.meta;
        L.mr[l] = mr;
        L.irrev[l] = irrev ? 1u : 0u;
    } else if (RR == 1) {
        if (pre) rep_prefetch(h, s, pr);
        const u32 x0 = philox_x0(C.seed, (u32)i, d);
        if (C.rtable) ra = C.racts[scale_rank(x0, C.rtotal)];
        L.x0[l] = x0;
    } else if (RR == 2) {
        L.valid[1][l] = quick_safe(s, a) ? 1u : 0u;
    } else {
        L.valid[0][l] = quick_pseudo(s, a) ? 1u : 0u;
    }
    PST(0);
    pair_barrier();
    PST(1);

    // ---- phase 1
    if (RR == 2) __builtin_amdgcn_s_setprio(0);
    const bool valid = (L.valid[0][l] & L.valid[1][l]) != 0;
    const bool mv = pre && valid;  // env_ply runs
    Pos ns = s;                    // the position generated for: post-move, or s itself
    ns.meta = (ns.meta & ~(u32)M_RIGHTS) | eff_rights(s);
    if (mv) {
        ns.k = L.ns[0][l]; ns.q = L.ns[1][l]; ns.r = L.ns[2][l]; ns.b = L.ns[3][l];
        ns.n = L.ns[4][l]; ns.p = L.ns[5][l]; ns.w = L.ns[6][l];
        ns.meta = L.nmeta[l];
    }
    Gen g;
    gen_base(ns, g);
    if (RR == 0) {
        gen_pins(ns, g);
        L.pin3[0][l] = g.checkmask;
        L.pin3[1][l] = g.pinned;
        L.pin3[2][l] = g.pinrays;
        L.f0[l] = g.in_check ? 1u : 0u;
    } else if (RR == 1) {
        L.f1[l] = (mv && mover_checked(s, ns, white, a)) ? 1u : 0u;
    } else if (RR == 2) {
        L.enemy[1][l] = g.ks >= 0 ? side_attacks_leapers(ns, !g.white) | side_attacks_orth(ns, !g.white) : 0ull;
    } else {
        L.enemy[2][l] = g.ks >= 0 ? side_attacks_diag(ns, !g.white) : 0ull;
    }
    u64* const mrow = out.mask ? out.mask + ii : nullptr;
    PST(2);
    pair_barrier();
    PST(3);

    // ---- phase 2
    const bool opp_chk = L.f0[l] != 0, my_chk = L.f1[l] != 0;
    const bool both = mv && opp_chk && my_chk;  // lib.rs:1442-1446: the move is void
    const bool gen = live && !both;             // the next side's moves (of ns) are due
    const bool big = popc(g.own) > SCRATCH_SLOTS;
    g.in_check = opp_chk;
    if (RR != 0) {
        g.checkmask = L.pin3[0][l];
        g.pinned = L.pin3[1][l];
        g.pinrays = L.pin3[2][l];
    }
    g.enemy_att = L.enemy[1][l] | L.enemy[2][l];
    MoveSet ms;
    moveset_clear(ms);
    int part = 0;
    if (RR == 0) {  // castles (counted here), pawns: the fast ones' targets parked as well
        gen_castles(ns, g);
        if (gen && !big) {
            part = gen_pawns(ns, g, ms, scr) + popc(g.castles);
            for (u64 fp = ms.fastp; fp; fp &= fp - 1) {
                const int sq = ctz(fp);
                scr.put(ordinal(g.own, sq), fast_pawn_targets(ms, sq, g.white));
            }
        }
        L.cbw[0][0][l] = scr.c0;
        L.cbw[0][1][l] = scr.c1;
        L.castles[l] = g.castles;
        L.part[0][l] = (u32)part;
    } else if (RR == 1) {  // knights, kings (while the probe lands), the 3-fold commit
        if (gen && !big) {
            part = gen_knights(ns, g, ms, scr) + gen_kings(ns, g, ms, scr);
        }
        L.cbw[1][0][l] = scr.c0;
        L.cbw[1][1][l] = scr.c1;
        L.part[1][l] = (u32)part;
        int c = 0;
        u32 hl = hl_of(s.meta);
        if (mv && !both) {
            pin(pr.e0.hdr); pin(pr.e0.k); pin(pr.e0.q); pin(pr.e0.r);
            pin(pr.e0.b); pin(pr.e0.n); pin(pr.e0.p); pin(pr.e0.w);
            c = rep_commit(h, s, pr, hl, L.irrev[l] != 0);  // table write deferred to h.commit()
        }
        L.rep[l] = (u32)c | (hl << 8);
        L.ra[l] = ra;
    } else if (RR == 2) {  // queens, bishops
        if (gen && !big) {
            part = gen_sliders<QUEEN>(ns, g, ms, scr);
        }
        L.cbw[2][0][l] = scr.c0;
        L.cbw[2][1][l] = scr.c1;
        L.part[2][l] = (u32)part;
    } else {  // rooks; a big board's whole count
        if (gen && !big) {
            part = gen_sliders<ROOK>(ns, g, ms, scr) + gen_sliders<BISHOP>(ns, g, ms, scr);
        } else if (gen) {
            gen_castles(ns, g);
            part = count_legal(ns, g);
        }
        L.cbw[3][0][l] = scr.c0;
        L.cbw[3][1][l] = scr.c1;
        L.part[3][l] = (u32)part;
    }
    PST(4);
    pair_barrier();
    PST(5);

    // ---- phase 3: the outcome (every role: identical arithmetic)
    if (RR == 0) __builtin_amdgcn_s_setprio(0);
    if (RR == 2) __builtin_amdgcn_s_setprio(2);  // the pick: this phase's longest chain
    const int total = gen ? (int)(L.part[0][l] + L.part[1][l] + L.part[2][l] + L.part[3][l]) : 0;
    const u32 rpk = L.rep[l];
    const int c = (int)(rpk & 0xFFu);
    const u32 hl = rpk >> 8;
    StepOut o = {0, 0, R_NONE, 0};
    Pos fs = s;  // the state after the step
    if (!valid) {
        o.reward = -10;
        o.done = done0 ? 1 : 0;
        o.reason = R_INVALID;
    } else if (done0) {
        o.done = 1;
        o.reason = R_DONE_ALREADY;
    } else if (cap) {
        o.done = 1;
        o.reason = R_MOVE_CAP;
    } else if (both) {
        o.done = 1;
        o.reason = R_BOTH_CHECKED;
    } else {
        const u32 chk = white ? ((my_chk ? M_WCHK : 0u) | (opp_chk ? M_BCHK : 0u))
                              : ((opp_chk ? M_WCHK : 0u) | (my_chk ? M_BCHK : 0u));
        fs = ns;
        fs.meta = with_hl((ns.meta & ~(u32)(M_WCHK | M_BCHK | M_DONE)) | chk | ((c >= 3 || c == 0) ? M_DONE : 0u), hl);
        o.reward = -10 + (RR == 1 ? (int)L.mr[l] : 0);  // INVALID_ACTION_REWARD + move reward (Q9; Q1 reports it)
        o.moved = 1;
        if (c >= 3) { o.done = 1; o.reason = R_REPETITION; }
        if (c == 0) { o.done = 1; o.reason = R_WINDOW_FULL; }
        if (total == 0 && opp_chk) {  // 270-272
            fs.meta |= M_DONE;
            o.done = 1;
            o.reward += 100;
            o.reason = R_MATE;
        }
        if (!o.done && !white) fs.meta += (1u << M_MC_SHIFT);  // 291-292
    }
    const bool reset = live && autoreset && o.done;
    if (reset) fs = icd->pos;
    // boards outside the fast path (per-piece fallback): both kings checked (the pre-move
    // board regenerates), or more own pieces than slots
    const bool slow = live && !reset && (both || big);

    // this role's 16 mask rows (Q0: and the castles word)
    if (mrow && live) {
        if (reset) {
            const u64 iown = icd->own;
#pragma unroll
            for (int k = 0; k < 16; k++) {
                const int sq = 16 * RR + k;
                const u64 w = ((iown >> sq) & 1) ? icd->slots[popc(iown & below(sq))] : 0ull;
                apiq_store(mrow + sq * N, w);
            }
        } else if (slow) {
            apiq_slow_rows<RR>(fs, mrow, N);
        } else {  // every own piece's targets are parked (pawns too): one LDS read per row
            int j = popc(g.own & below(16 * RR));
#pragma unroll
            for (int k = 0; k < 16; k++) {
                const int sq = 16 * RR + k;
                const bool own = (g.own >> sq) & 1;
                const u64 w = scr.get(j & (SCRATCH_SLOTS - 1));
                apiq_store(mrow + sq * N, own ? w : 0ull);
                j += own ? 1 : 0;
            }
        }
        if (RR == 0) {
            const u32 cs = reset ? icd->castles : slow ? apiq_slow_castles(fs) : L.castles[l];
            const bool cwh = reset ? icd->white != 0 : slow ? (fs.meta & M_WHITE) != 0 : g.white;
            u64 cwd = 0;
            if (cs & 1) cwd |= cwh ? (1ull << 1) : (1ull << 3);  // QS: 4097 / 4099
            if (cs & 2) cwd |= cwh ? (1ull << 0) : (1ull << 2);  // KS: 4096 / 4098
            mrow[64 * N] = cwd;
        }
    }
#ifdef GC_PSTAMPS
    const unsigned long long pst_rt1 = __builtin_amdgcn_s_memrealtime();
#endif
    if (live && RR == 2) {  // the pick (action-id order: the mask's), the count, the env's next action
        int tot = total;
        uint16_t p = (uint16_t)A_NONE;
        if (reset) {
            tot = (int)C.rtotal;
            p = (uint16_t)L.ra[l];  // (the quads run only with the start position's table)
        } else if (slow) {
            const u32 r = apiq_slow_pick(fs, L.x0[l]);
            tot = (int)(r >> 16);
            p = (uint16_t)(r & 0xFFFFu);
        } else if (tot > 0) {  // castles last (KS 4096 / 4098 before QS 4097 / 4099)
            const u32 cs = L.castles[l];
            const int normal = tot - popc(cs);
            int k = (int)scale_rank(L.x0[l], (u32)tot);
            if (k < normal) {
                p = (uint16_t)ord_pick(scr, g.own, L.cbw[0][0][l] | L.cbw[1][0][l] | L.cbw[2][0][l] | L.cbw[3][0][l],
                                       L.cbw[0][1][l] | L.cbw[1][1][l] | L.cbw[2][1][l] | L.cbw[3][1][l], normal, k);
            } else {
                k -= normal;
                p = (cs & 2) && k == 0 ? (uint16_t)(g.white ? A_KSW : A_KSB) : (uint16_t)(g.white ? A_QSW : A_QSB);
            }
        }
        if (out.cnt) out.cnt[i] = tot;
        if (out.pick) {
            const PairIO io = store_io(slab, nn);
            d += tot > 0 ? 1u : 0u;
            out.pick[i] = p;
            io.act[i] = p;
            io.draw[i] = d;
        }
    } else if (live && RR == 3) {
        if (out.obs) WRITE_OBS_Q3(fs, out.obs, i, nn);
    } else if (live && RR == 1) {
        if (reset) h.bump_gen();
        out.rw[i] = o.reward;
        out.dn[i] = (uint8_t)o.done;
        out.rs[i] = (uint8_t)o.reason;
        h.commit();
        const PairIO io = store_io(slab, nn);
        io.store(i, fs);
        h.flush(g0);
        io.nsteps[i] = nst + 1;
        io.reward[i] = o.reward;
        io.done[i] = (uint8_t)o.done;
        io.reason[i] = (uint8_t)o.reason;
    }
#ifdef GC_PSTAMPS
    PST(6);
    if (g_pst_out != nullptr && l == 0) {  // (tools/api_pstamp_probe.py)
        const size_t w = (size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
        for (int k = 0; k < 8; k++) g_pst_out[w * 12 + k] = gc_pst[threadIdx.x >> 6][k];
        g_pst_out[w * 12 + 8] = pst_entry;
        g_pst_out[w * 12 + 9] = pst_rt0;
        g_pst_out[w * 12 + 10] = pst_rt1;
        g_pst_out[w * 12 + 11] = __builtin_amdgcn_s_memrealtime();
    }
#endif
}

// 16 argument dwords, as k_env_step_api4 (all preloaded)
__global__ void __launch_bounds__(4 * QUAD_BOARDS * QUADS_WG) __attribute__((amdgpu_waves_per_eu(4)))
    k_env_step_api4(uint8_t* __restrict__ slab, uint64_t seed, u64* __restrict__ htab,
                    const uint16_t* __restrict__ racts, const EnvDev::InitCache* __restrict__ icd,
                    const uint16_t* __restrict__ acts, const ApiOut* __restrict__ outp, int nn,
                    u32 rinfo /* autoreset << 17 | ic.table << 16 | ic.total */) {
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int qw = wv >> 2;
    const int role = (wv & 3) ^ ((qw & 1) ? GC_QXOR : 0);  // as k_env_rollout4: every SIMD a stateful + a stateless role
    const int l = threadIdx.x & (QUAD_BOARDS - 1);
    const int i = (blockIdx.x * QUADS_WG + qw) * QUAD_BOARDS + l;
    ApiOut out = *outp;
    asm volatile("" : "+s"(out.rw), "+s"(out.dn), "+s"(out.rs), "+s"(out.mask), "+s"(out.obs), "+s"(out.cnt),
                 "+s"(out.pick), "+s"(out.ms));
    switch (role) {
        case 0: apiq_run<0>(slab, seed, htab, racts, icd, acts, out, nn, rinfo, qw, l, i); break;
        case 1: apiq_run<1>(slab, seed, htab, racts, icd, acts, out, nn, rinfo, qw, l, i); break;
        case 2: apiq_run<2>(slab, seed, htab, racts, icd, acts, out, nn, rinfo, qw, l, i); break;
        default: apiq_run<3>(slab, seed, htab, racts, icd, acts, out, nn, rinfo, qw, l, i); break;
    }
}

// ----------------------------------------------------------------------------- API step, quads, random opponent
// k_env_step_api2_vs<false>'s contract (a WHITE agent against the random opponent: the agent's
// validated action, the reply inside the step, chess_v2.py:219-294 with opponent_policy set) on
// four waves per 64 boards.  The agent's ply runs as k_env_step_api4's
// phases 0-2 with the opponent's moves made as the rollout's move sets; the reply is picked and
// applied in phase 3; phases 4-6 are k_env_step_api4's phases 1-3 for the position the mask
// describes -- the reply played, or (no reply) the state after the agent's half as it stands:
//
//   phase 0   Q0: applies the agent's action              Q1: its window probe, two Philox words
//             Q2, Q3: validate it (quick_safe / quick_pseudo)     and the reset table's picks
//   phase 1   the opponent's position: Q0 pins, Q1 the agent's own check, Q2 / Q3 the enemy map
//   phase 2   Q0 castles, pawn and knight sets | Q1 the agent ply's 3-fold commit
//             Q2 rook / queen direction sets, king sets | Q3 bishop / queen ones
//   phase 3   every role: the agent ply's outcome (same arithmetic from LDS); Q2 picks the reply
//             (draw d, move-set order) and applies it; Q1 writes the agent ply's window entry and
//             probes the pre-reply board
//   phase 4   the mask's position: Q0 pins, Q1 the opponent's own check, Q2 / Q3 the enemy map
//   phase 5   Q0 castles, pawns | Q1 knights, kings, the reply's 3-fold commit | Q2 queens
//             Q3 rooks, bishops (pieces parked by ordinal, as k_env_step_api4)
//   phase 6   every role: the reply's outcome, its 16 mask rows; Q2 the agent's pick (the next
//             draw, action-id order), count and next action; Q3 the observation; Q1 the outputs,
//             the state and the window
//
// Same draws in the same order as k_env_step_api2_vs (and the one-wave k_env_step_api<true>).
// A BLACK agent (whose reset opens with the opponent's move) stays on k_env_step_api2_vs<true>.
struct ApiQvSetCounts {
    u64 cwx[2][4][QUAD_BOARDS];  // Q2 / Q3 -> Q2: their sets' byte counts (phase 2)
    u64 cw0[QUAD_BOARDS];        // Q0 -> Q2: its sets' (words 0, 1: pawns, knights)
    u64 cw1[QUAD_BOARDS];
};
struct ApiQuadVsLds {
    union {
        u64 sets[SW_SETS][QUAD_BOARDS];         // phases 2-3: the opponent's move sets
        u64 slots[SCRATCH_SLOTS][QUAD_BOARDS];  // phases 5-6: parked targets per own-piece ordinal
    };
    u64 ns[NBB][QUAD_BOARDS];    // Q0 -> all (phase 0): the agent's post-move board
    u32 nmeta[QUAD_BOARDS];
    int32_t mr[QUAD_BOARDS];     //   its capture reward
    u32 irrev[QUAD_BOARDS];      //   irreversible move
    u64 ns2[NBB][QUAD_BOARDS];   // Q2 -> all (phase 3): the mask's position (the reply played, or the kept state)
    u32 nmeta2[QUAD_BOARDS];
    int32_t mr2[QUAD_BOARDS];    //   the reply's capture reward
    u32 irrev2[QUAD_BOARDS];
    u32 oa[QUAD_BOARDS];         // Q2 -> Q1: the reply
    u32 valid[2][QUAD_BOARDS];   // Q3 ([0]: the move's shape), Q2 ([1]: king safety) -> all
    u64 pin3[3][QUAD_BOARDS];    // Q0 -> Q2, Q3: check mask, pinned, pin rays (phases 1 and 4)
    u32 f0[QUAD_BOARDS];         // Q0 -> all: the side to move is in check
    u64 enemy[3][QUAD_BOARDS];   // Q2 ([1]), Q3 ([2]) -> all: the enemy map's parts
    u32 f1[QUAD_BOARDS];         // Q1 -> all: the mover is in check after its move
    union {
        ApiQvSetCounts sc;                  // phases 2-3
        u64 cbw[4][2][QUAD_BOARDS];         // phases 5-6: per role, its pieces' move counts by ordinal
    };
    u32 part[4][QUAD_BOARDS];    // move totals (Q0's holds the castles; phase 5: Q3's a big board's)
    u32 castles[QUAD_BOARDS];    // Q0 -> all
    u32 rep[QUAD_BOARDS];        // Q1 -> all: the agent ply's 3-fold count | window length << 8
    u32 rep2[QUAD_BOARDS];       // Q1 -> all: the reply's
    u32 x0[QUAD_BOARDS];         // Q1 -> Q2: the Philox words of draws d, d + 1
    u32 x1[QUAD_BOARDS];
    u32 x2[QUAD_BOARDS];         // (BLACK: d + 2, after a reply and a reset's opening)
    u32 ra[2][QUAD_BOARDS];      // Q1 -> all: the table picks for x0 / x1 (WHITE: a reset board's pick; BLACK: the opening)
};
__shared__ ApiQuadVsLds g_apiqv_lds[QUADS_WG];

template <int RR, bool BLACK>
__device__ __forceinline__ void apiqv_run(uint8_t* __restrict__ slab, uint64_t seed, u64* __restrict__ htab,
                                          const uint16_t* __restrict__ racts, const EnvDev::InitCache* __restrict__ icd,
                                          const uint16_t* __restrict__ acts, const ApiOut& out, int nn, u32 rinfo,
                                          int qw, int l, int i) {
    ApiQuadVsLds& L = g_apiqv_lds[qw];
#ifdef GC_PSTAMPS  // (tools/api_pstamp_probe.py vs: segments 0-6 = the phases' work, 7 = entry loads + barrier waits)
    const unsigned long long pst_entry = __builtin_amdgcn_s_memrealtime();
    if (l == 0) {
        for (int k = 0; k < 8; k++) gc_pst[threadIdx.x >> 6][k] = 0;
        gc_pst[threadIdx.x >> 6][8] = __builtin_amdgcn_s_memtime();
    }
#endif
    const int autoreset = (rinfo >> 17) & 1;
    rinfo &= 0x1FFFFu;
    const bool live = i < nn;
    const int ii = live ? i : nn - 1;  // dead lanes read a valid board, store nothing
    const size_t N = out.ms;           // the mask rows' stride
    const PairIO in_io(slab, nn);
    const PairCtx C = {seed, htab, in_io.hgen, racts, icd, (rinfo >> 16) != 0, rinfo & 0xFFFFu};
    Pos s = in_io.load(ii);
    u32 ua = acts[ii], g0 = 0, nst = 0, d = 0;
    if (RR == 1) { g0 = in_io.hgen[ii]; nst = in_io.nsteps[ii]; }
    if (RR == 1 || RR == 2) d = in_io.draw[ii];
    pin(s); pin(ua); pin(g0); pin(nst); pin(d);
    PST(7);
#ifdef GC_PSTAMPS
    const unsigned long long pst_rt0 = __builtin_amdgcn_s_memrealtime();
#endif
    const int a = (int)ua;
    DevHist h = DevHist{htab, in_io.hgen, g0, ii, BLACK ? HTAB_BITS_UNCAPPED : HTAB_BITS};
    if (BLACK && RR == 1) h.sp = icd->spill;  // a BLACK agent's windows may spill
    OrdScratch scr{&L.slots[0][l], 0ull, 0ull};
    // (Q3 over Q1 in phases 0, 5 and 6, where Q3's chain is the longer: 20.9 vs 20.7 us per launch)
    if (RR != 3) __builtin_amdgcn_s_setprio(2);
    const bool done0 = (s.meta & M_DONE) != 0;   // chess_v2.py:245-251
    const bool cap = mc_of(s.meta) > MOVES_MAX;  // 252-258
    const bool white = (s.meta & M_WHITE) != 0;  // the agent's colour
    const bool pre = live && !done0 && !cap;

    // ---- phase 0: the agent's action applied (speculatively) and validated; Q1's loads issued
    RepProbe pr;
    uint16_t ra0 = (uint16_t)A_NONE, ra1 = (uint16_t)A_NONE;
    if (RR == 0) {
        Pos ns = s;
        ns.meta = (ns.meta & ~(u32)M_RIGHTS) | eff_rights(s);  // State::new
        int mr = 0;
        bool irrev = false;
        apply_legal(ns, white, a, &mr, &irrev);
        L.ns[0][l] = ns.k; L.ns[1][l] = ns.q; L.ns[2][l] = ns.r; L.ns[3][l] = ns.b;
        L.ns[4][l] = ns.n; L.ns[5][l] = ns.p; L.ns[6][l] = ns.w;
        L.nmeta[l] = ns.meta;
        L.mr[l] = mr;
        L.irrev[l] = irrev ? 1u : 0u;
    } else if (RR == 1) {
        if (pre) rep_prefetch(h, s, pr);
        const u32 x0 = philox_x0(C.seed, (u32)i, d), x1 = philox_x0(C.seed, (u32)i, d + 1);
        // WHITE: a reset board's pick in action-id order; BLACK: the opponent's opening after a
        // reset, in move-set order (chess_v2.py:208-216), for the draw it would take
        const uint16_t* const tab = BLACK ? C.racts + RESET_ACTS_MAX : C.racts;
        if (C.rtable) {
            ra0 = tab[scale_rank(x0, C.rtotal)];
            ra1 = tab[scale_rank(x1, C.rtotal)];
        }
        L.x0[l] = x0;
        L.x1[l] = x1;
        if (BLACK) L.x2[l] = philox_x0(C.seed, (u32)i, d + 2);
    } else if (RR == 2) {
        L.valid[1][l] = quick_safe(s, a) ? 1u : 0u;
    } else {
        L.valid[0][l] = quick_pseudo(s, a) ? 1u : 0u;
    }
    PST(0);
    pair_barrier();
    PST(7);

    // ---- phase 1: the opponent's position
    if (RR == 2) __builtin_amdgcn_s_setprio(0);
    const bool valid = (L.valid[0][l] & L.valid[1][l]) != 0;
    const bool mv = pre && valid;  // the agent's env_ply runs
    Pos ns = s;
    ns.meta = (ns.meta & ~(u32)M_RIGHTS) | eff_rights(s);
    if (mv) {
        ns.k = L.ns[0][l]; ns.q = L.ns[1][l]; ns.r = L.ns[2][l]; ns.b = L.ns[3][l];
        ns.n = L.ns[4][l]; ns.p = L.ns[5][l]; ns.w = L.ns[6][l];
        ns.meta = L.nmeta[l];
    }
    Gen g;
    gen_base(ns, g);
    if (RR == 0) {
        gen_pins(ns, g);
        L.pin3[0][l] = g.checkmask;
        L.pin3[1][l] = g.pinned;
        L.pin3[2][l] = g.pinrays;
        L.f0[l] = g.in_check ? 1u : 0u;
    } else if (RR == 1) {
        L.f1[l] = (mv && mover_checked(s, ns, white, a)) ? 1u : 0u;
    } else if (RR == 2) {
        L.enemy[1][l] = g.ks >= 0 ? side_attacks_leapers(ns, !g.white) | side_attacks_orth(ns, !g.white) : 0ull;
    } else {
        L.enemy[2][l] = g.ks >= 0 ? side_attacks_diag(ns, !g.white) : 0ull;
    }
    PST(1);
    pair_barrier();
    PST(7);

    // ---- phase 2: the opponent's move sets (as the rollout's quads); Q1 the agent ply's commit
    const bool opp_chk = L.f0[l] != 0, my_chk = L.f1[l] != 0;
    const bool both = mv && opp_chk && my_chk;  // lib.rs:1442-1446: the move is void
    const bool gen = mv && !both;               // the opponent's moves are due
    g.in_check = opp_chk;
    if (RR != 0) {
        g.checkmask = L.pin3[0][l];
        g.pinned = L.pin3[1][l];
        g.pinrays = L.pin3[2][l];
    }
    g.enemy_att = L.enemy[1][l] | L.enemy[2][l];
    QuadSetsT<ApiQuadVsLds> Q{L, l, {0, 0, 0, 0}, 0};
    const int mr = L.mr[l];
    const bool irrev = L.irrev[l] != 0;
    if (RR == 0) {
        gen_castles(ns, g);
        if (gen) {
            u64 T[SW_SETS];
            sw_pawns(ns, g, T);
            Q.put_all<SW_P1, SW_N>(T + SW_P1);
            sw_knights(ns, g, T);
            Q.put_all<SW_N, SW_ORTH>(T + SW_N);
            Q.part += popc(g.castles);
        }
        L.sc.cw0[l] = Q.cw[0];
        L.sc.cw1[l] = Q.cw[1];
        L.castles[l] = g.castles;
        L.part[0][l] = (u32)Q.part;
    } else if (RR == 1) {
        int c = 0;
        u32 hl = hl_of(s.meta);
        if (gen) {
            pin(pr.e0.hdr); pin(pr.e0.k); pin(pr.e0.q); pin(pr.e0.r);
            pin(pr.e0.b); pin(pr.e0.n); pin(pr.e0.p); pin(pr.e0.w);
            c = rep_commit(h, s, pr, hl, irrev);  // table write deferred to h.commit()
        }
        L.rep[l] = (u32)c | (hl << 8);
        L.ra[0][l] = ra0;
        L.ra[1][l] = ra1;
    } else if (RR == 2) {  // unconditional: ignored unless the opponent's moves are due
        u64 T[SW_SETS];
        sw_orth(ns, g, T);
        Q.put_all<SW_ORTH, SW_DIAG>(T + SW_ORTH);
        sw_kings(ns, g, T);
        Q.put_all<SW_K, SW_SETS>(T + SW_K);
        L.part[2][l] = (u32)Q.part;
#pragma unroll
        for (int k = 0; k < 4; k++) L.sc.cwx[0][k][l] = Q.cw[k];
    } else {
        u64 T[SW_SETS];
        sw_diag(ns, g, T);
        Q.put_all<SW_DIAG, SW_K>(T + SW_DIAG);
        L.part[3][l] = (u32)Q.part;
#pragma unroll
        for (int k = 0; k < 4; k++) L.sc.cwx[1][k][l] = Q.cw[k];
    }
    PST(2);
    pair_barrier();
    PST(7);

    // ---- phase 3: the agent ply's outcome (k_env_step_api2_vs half A); Q2 picks and plays the reply
    if (RR == 0) __builtin_amdgcn_s_setprio(0);
    if (RR == 2) __builtin_amdgcn_s_setprio(2);
    const int tot_opp = gen ? (int)(L.part[0][l] + L.part[2][l] + L.part[3][l]) : 0;
    StepOut o = {0, 0, R_NONE, 0};
    bool cont = false;  // the opponent replies
    Pos s1 = s;         // the state after the agent's half
    {
        const u32 rpk = L.rep[l];
        const int c = (int)(rpk & 0xFFu);
        const u32 hl = rpk >> 8;
        if (!valid) {
            o.reward = -10;
            o.done = done0 ? 1 : 0;
            o.reason = R_INVALID;
        } else if (done0) {
            o.done = 1;
            o.reason = R_DONE_ALREADY;
        } else if (cap) {
            o.done = 1;
            o.reason = R_MOVE_CAP;
        } else if (both) {
            o.done = 1;
            o.reason = R_BOTH_CHECKED;
        } else {
            const u32 chk = white ? ((my_chk ? M_WCHK : 0u) | (opp_chk ? M_BCHK : 0u))
                                  : ((opp_chk ? M_WCHK : 0u) | (my_chk ? M_BCHK : 0u));
            s1 = ns;
            s1.meta = with_hl((ns.meta & ~(u32)(M_WCHK | M_BCHK | M_DONE)) | chk | ((c >= 3 || c == 0) ? M_DONE : 0u), hl);
            o.reward = -10 + mr;  // Q9
            o.moved = 1;
            if (c >= 3) { o.done = 1; o.reason = R_REPETITION; }
            if (c == 0) { o.done = 1; o.reason = R_WINDOW_FULL; }
            if (tot_opp == 0 && opp_chk) {  // 270-272
                s1.meta |= M_DONE;
                o.done = 1;
                o.reward += 100;
                o.reason = R_MATE;
            }
            if (!o.done && tot_opp == 0) {  // 120-122: the opponent's policy "resigns"
                s1.meta |= M_DONE;
                o.done = 1;
                o.reason = R_OPP_NO_MOVE;
            }
            cont = !o.done;
        }
    }
    if (RR == 2) {  // the reply (move-set order, draw d) played on the state after the agent's half
        Pos p = s1;
        p.meta = (p.meta & ~(u32)M_RIGHTS) | eff_rights(s1);
        int mr2 = 0;
        bool irrev2 = false;
        int oa = A_NONE;
        if (cont) {
            u64 cw[4];
#pragma unroll
            for (int k = 0; k < 4; k++) cw[k] = Q.cw[k] | L.sc.cwx[1][k][l];
            cw[0] |= L.sc.cw0[l];
            cw[1] |= L.sc.cw1[l];
            g.castles = L.castles[l];
            oa = sw_pick_lds(L, l, g, cw, tot_opp, (int)scale_rank(L.x0[l], (u32)tot_opp));
            apply_legal(p, (s1.meta & M_WHITE) != 0, oa, &mr2, &irrev2);
        }
        L.ns2[0][l] = p.k; L.ns2[1][l] = p.q; L.ns2[2][l] = p.r; L.ns2[3][l] = p.b;
        L.ns2[4][l] = p.n; L.ns2[5][l] = p.p; L.ns2[6][l] = p.w;
        L.nmeta2[l] = p.meta;
        L.mr2[l] = mr2;
        L.irrev2[l] = irrev2 ? 1u : 0u;
        L.oa[l] = (u32)oa;
    } else if (RR == 1 && live) {
        h.commit();  // the agent ply's window write lands before the reply probes the table
        if (cont) rep_prefetch(h, s1, pr);
    }
    PST(3);
    pair_barrier();
    PST(7);

    // ---- phase 4: the mask's position (the agent to move after a reply)
    if (RR == 0) __builtin_amdgcn_s_setprio(2);
    if (RR == 2) __builtin_amdgcn_s_setprio(0);
    Pos P;
    P.k = L.ns2[0][l]; P.q = L.ns2[1][l]; P.r = L.ns2[2][l]; P.b = L.ns2[3][l];
    P.n = L.ns2[4][l]; P.p = L.ns2[5][l]; P.w = L.ns2[6][l];
    P.meta = L.nmeta2[l];
    gen_base(P, g);
    if (RR == 0) {
        gen_pins(P, g);
        L.pin3[0][l] = g.checkmask;
        L.pin3[1][l] = g.pinned;
        L.pin3[2][l] = g.pinrays;
        L.f0[l] = g.in_check ? 1u : 0u;
    } else if (RR == 1) {
        L.f1[l] = (cont && mover_checked(s1, P, (s1.meta & M_WHITE) != 0, (int)L.oa[l])) ? 1u : 0u;
    } else if (RR == 2) {
        L.enemy[1][l] = g.ks >= 0 ? side_attacks_leapers(P, !g.white) | side_attacks_orth(P, !g.white) : 0ull;
    } else {
        L.enemy[2][l] = g.ks >= 0 ? side_attacks_diag(P, !g.white) : 0ull;
    }
    PST(4);
    pair_barrier();
    PST(7);

    // ---- phase 5: the mask position's moves, parked by ordinal; Q1 the reply's commit
    const bool chk2 = L.f0[l] != 0, mchk2 = L.f1[l] != 0;  // the agent in check; the opponent, after its reply
    const bool both2 = cont && chk2 && mchk2;
    const bool gen2 = live && !both2;
    const bool big = popc(g.own) > SCRATCH_SLOTS;
    g.in_check = chk2;
    if (RR != 0) {
        g.checkmask = L.pin3[0][l];
        g.pinned = L.pin3[1][l];
        g.pinrays = L.pin3[2][l];
    }
    g.enemy_att = L.enemy[1][l] | L.enemy[2][l];
    MoveSet ms;
    moveset_clear(ms);
    int part = 0;
    if (RR == 0) {  // castles (counted here), pawns: the fast ones' targets parked as well
        gen_castles(P, g);
        if (gen2 && !big) {
            part = gen_pawns(P, g, ms, scr) + popc(g.castles);
            for (u64 fp = ms.fastp; fp; fp &= fp - 1) {
                const int sq = ctz(fp);
                scr.put(ordinal(g.own, sq), fast_pawn_targets(ms, sq, g.white));
            }
        }
        L.cbw[0][0][l] = scr.c0;
        L.cbw[0][1][l] = scr.c1;
        L.castles[l] = g.castles;
        L.part[0][l] = (u32)part;
    } else if (RR == 1) {  // knights, kings (while the probe lands), the reply's 3-fold commit
        if (gen2 && !big) part = gen_knights(P, g, ms, scr) + gen_kings(P, g, ms, scr);
        L.cbw[1][0][l] = scr.c0;
        L.cbw[1][1][l] = scr.c1;
        L.part[1][l] = (u32)part;
        int c = 0;
        u32 hl = hl_of(s1.meta);
        if (cont && !both2) {
            pin(pr.e0.hdr); pin(pr.e0.k); pin(pr.e0.q); pin(pr.e0.r);
            pin(pr.e0.b); pin(pr.e0.n); pin(pr.e0.p); pin(pr.e0.w);
            c = rep_commit(h, s1, pr, hl, L.irrev2[l] != 0);  // table write deferred to h.commit()
        }
        L.rep2[l] = (u32)c | (hl << 8);
    } else if (RR == 2) {  // queens
        if (gen2 && !big) part = gen_sliders<QUEEN>(P, g, ms, scr);
        L.cbw[2][0][l] = scr.c0;
        L.cbw[2][1][l] = scr.c1;
        L.part[2][l] = (u32)part;
    } else {  // rooks, bishops; a big board's whole count
        if (gen2 && !big) {
            part = gen_sliders<ROOK>(P, g, ms, scr) + gen_sliders<BISHOP>(P, g, ms, scr);
        } else if (gen2) {
            gen_castles(P, g);
            part = count_legal(P, g);
        }
        L.cbw[3][0][l] = scr.c0;
        L.cbw[3][1][l] = scr.c1;
        L.part[3][l] = (u32)part;
    }
    PST(5);
    pair_barrier();
    PST(7);

    // ---- phase 6: the reply's outcome (k_env_step_api2_vs half B), the mask rows, the outputs
    if (RR == 0) __builtin_amdgcn_s_setprio(0);
    if (RR == 2) __builtin_amdgcn_s_setprio(2);
    const int total = gen2 ? (int)(L.part[0][l] + L.part[1][l] + L.part[2][l] + L.part[3][l]) : 0;
    Pos fs = s1;         // the state after the step
    bool alone = false;  // the state stays (the reply left both kings checked): its moves were not made
    if (cont) {
        if (both2) {  // the engine raises, the env ends
            o.reason = R_BOTH_CHECKED;
            o.done = 1;
            alone = true;
        } else {
            const u32 rpk = L.rep2[l];
            const int c = (int)(rpk & 0xFFu);
            const u32 hl = rpk >> 8;
            const bool ow = (s1.meta & M_WHITE) != 0;  // the opponent's colour
            const u32 chk = ow ? ((mchk2 ? M_WCHK : 0u) | (chk2 ? M_BCHK : 0u))
                               : ((chk2 ? M_WCHK : 0u) | (mchk2 ? M_BCHK : 0u));
            fs = P;
            fs.meta = with_hl((P.meta & ~(u32)(M_WCHK | M_BCHK | M_DONE)) | chk | ((c >= 3 || c == 0) ? M_DONE : 0u), hl);
            o.reward -= (int)L.mr2[l];  // 283
            if (c >= 3) { o.done = 1; o.reason = R_REPETITION; }
            if (c == 0) { o.done = 1; o.reason = R_WINDOW_FULL; }
            if (total == 0 && chk2) {  // 285-288
                fs.meta |= M_DONE;
                o.done = 1;
                o.reward -= 100;
                o.reason = R_MATED;
            }
            if (fs.meta & M_WHITE) fs.meta += (1u << M_MC_SHIFT);  // 291-292
        }
    }
    const bool reset = live && autoreset && o.done;  // chess_v2.py:183-206
    u32 nd = cont ? 1u : 0u;                         // draws taken by the reply (and the opening)
    if (reset) fs = icd->pos;
    const OpenCache* oc = nullptr;  // BLACK, a reset: the position after the opening
    if (BLACK && reset) {  // the opponent opens as WHITE (208-216): the opening of draw nd, settled beforehand
        oc = icd->open + scale_rank(nd == 0 ? L.x0[l] : L.x1[l], C.rtotal);
        if (RR == 1) {  // the window: the reply's write, the reset's new generation, the opening's entry
            h.commit();
            h.bump_gen();
            RepProbe po;
            rep_prefetch(h, fs, po);
            u32 hl = hl_of(fs.meta);
            (void)rep_commit(h, fs, po, hl, oc->irrev != 0);  // (count 1, length as the cache's)
        }
        fs = oc->pos;
        nd += 1;
    }
    // boards outside the fast path (per-piece fallback): the state kept after a void reply, more
    // own pieces than slots, or (BLACK) an opening's position with more own pieces than slots
    const bool slow = live && ((!reset && (alone || big)) || (BLACK && reset && !oc->usable));
    const bool cached = reset && !BLACK;  // the start position's rows, count and pick
    const bool ocached = BLACK && reset && oc->usable;  // the opening's
    u64* const mrow = out.mask ? out.mask + ii : nullptr;
    if (mrow && live) {
        if (cached || ocached) {
            const u64 iown = cached ? icd->own : oc->own;
            const u64* const islots = cached ? icd->slots : oc->slots;
#pragma unroll
            for (int k = 0; k < 16; k++) {
                const int sq = 16 * RR + k;
                const u64 w = ((iown >> sq) & 1) ? islots[popc(iown & below(sq))] : 0ull;
                apiq_store(mrow + sq * N, w);
            }
        } else if (slow) {
            apiq_slow_rows<RR>(fs, mrow, N);
        } else {  // every own piece's targets are parked (pawns too): one LDS read per row
            int j = popc(g.own & below(16 * RR));
#pragma unroll
            for (int k = 0; k < 16; k++) {
                const int sq = 16 * RR + k;
                const bool own = (g.own >> sq) & 1;
                const u64 w = scr.get(j & (SCRATCH_SLOTS - 1));
                apiq_store(mrow + sq * N, own ? w : 0ull);
                j += own ? 1 : 0;
            }
        }
        if (RR == 0) {
            const u32 cs = cached ? icd->castles : ocached ? oc->castles : slow ? apiq_slow_castles(fs) : L.castles[l];
            const bool cwh = cached ? icd->white != 0 : ocached ? oc->white != 0 : slow ? (fs.meta & M_WHITE) != 0 : g.white;
            u64 cwd = 0;
            if (cs & 1) cwd |= cwh ? (1ull << 1) : (1ull << 3);  // QS: 4097 / 4099
            if (cs & 2) cwd |= cwh ? (1ull << 0) : (1ull << 2);  // KS: 4096 / 4098
            mrow[64 * N] = cwd;
        }
    }
#ifdef GC_PSTAMPS
    const unsigned long long pst_rt1 = __builtin_amdgcn_s_memrealtime();  // the mask rows issued
#endif
    if (live && RR == 2) {  // the agent's pick (the next draw, action-id order), the count, the env's next action
        const u32 xp = nd == 0 ? L.x0[l] : nd == 1 ? L.x1[l] : L.x2[l];
        int tot = total;
        uint16_t p = (uint16_t)A_NONE;
        if (cached) {
            tot = (int)C.rtotal;
            p = (uint16_t)L.ra[nd][l];  // (the quads run only with the start position's table)
        } else if (ocached && oc->table) {
            tot = oc->total;
            p = icd->open_acts[(size_t)(oc - icd->open) * RESET_ACTS_MAX + scale_rank(xp, (u32)tot)];
        } else if (ocached) {  // (never with a standard start: more moves than the table holds)
            const u32 r = apiq_slow_pick(fs, xp);
            tot = (int)(r >> 16);
            p = (uint16_t)(r & 0xFFFFu);
        } else if (slow) {
            const u32 r = apiq_slow_pick(fs, xp);
            tot = (int)(r >> 16);
            p = (uint16_t)(r & 0xFFFFu);
        } else if (tot > 0) {  // castles last (KS 4096 / 4098 before QS 4097 / 4099)
            const u32 cs = L.castles[l];
            const int normal = tot - popc(cs);
            int k = (int)scale_rank(xp, (u32)tot);
            if (k < normal) {
                p = (uint16_t)ord_pick(scr, g.own, L.cbw[0][0][l] | L.cbw[1][0][l] | L.cbw[2][0][l] | L.cbw[3][0][l],
                                       L.cbw[0][1][l] | L.cbw[1][1][l] | L.cbw[2][1][l] | L.cbw[3][1][l], normal, k);
            } else {
                k -= normal;
                p = (cs & 2) && k == 0 ? (uint16_t)(g.white ? A_KSW : A_KSB) : (uint16_t)(g.white ? A_QSW : A_QSB);
            }
        }
        if (out.cnt) out.cnt[i] = tot;
        const PairIO io = store_io(slab, nn);
        u32 dn = d + nd;
        if (out.pick) {
            dn += tot > 0 ? 1u : 0u;
            out.pick[i] = p;
            io.act[i] = p;
        }
        io.draw[i] = dn;
    } else if (live && RR == 3) {
        if (out.obs) WRITE_OBS_Q3(fs, out.obs, i, nn);
    } else if (live && RR == 1) {
        if (reset && !BLACK) h.bump_gen();  // (BLACK: bumped before the opening's entry)
        out.rw[i] = o.reward;
        out.dn[i] = (uint8_t)o.done;
        out.rs[i] = (uint8_t)o.reason;
        h.commit();
        const PairIO io = store_io(slab, nn);
        io.store(i, fs);
        h.flush(g0);
        io.nsteps[i] = nst + 1;
        io.reward[i] = o.reward;
        io.done[i] = (uint8_t)o.done;
        io.reason[i] = (uint8_t)o.reason;
    }
#ifdef GC_PSTAMPS
    PST(6);
    if (g_pst_out != nullptr && l == 0) {
        const size_t w = (size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
        for (int k = 0; k < 8; k++) g_pst_out[w * 12 + k] = gc_pst[threadIdx.x >> 6][k];
        g_pst_out[w * 12 + 8] = pst_entry;
        g_pst_out[w * 12 + 9] = pst_rt0;
        g_pst_out[w * 12 + 10] = pst_rt1;
        g_pst_out[w * 12 + 11] = __builtin_amdgcn_s_memrealtime();
    }
#endif
}

// 16 argument dwords, as k_env_step_api2_vs (all preloaded)
template <bool BLACK>
__global__ void __launch_bounds__(4 * QUAD_BOARDS * QUADS_WG) __attribute__((amdgpu_waves_per_eu(4)))
    k_env_step_api4_vs(uint8_t* __restrict__ slab, uint64_t seed, u64* __restrict__ htab,
                       const uint16_t* __restrict__ racts, const EnvDev::InitCache* __restrict__ icd,
                       const uint16_t* __restrict__ acts, const ApiOut* __restrict__ outp, int nn,
                       u32 rinfo /* autoreset << 17 | ic.table << 16 | ic.total */) {
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int qw = wv >> 2;
    const int role = (wv & 3) ^ ((qw & 1) ? GC_QXOR : 0);  // as k_env_rollout4: every SIMD a stateful + a stateless role
    const int l = threadIdx.x & (QUAD_BOARDS - 1);
    const int i = (blockIdx.x * QUADS_WG + qw) * QUAD_BOARDS + l;
    ApiOut out = *outp;
    asm volatile("" : "+s"(out.rw), "+s"(out.dn), "+s"(out.rs), "+s"(out.mask), "+s"(out.obs), "+s"(out.cnt),
                 "+s"(out.pick), "+s"(out.ms));
    switch (role) {
        case 0: apiqv_run<0, BLACK>(slab, seed, htab, racts, icd, acts, out, nn, rinfo, qw, l, i); break;
        case 1: apiqv_run<1, BLACK>(slab, seed, htab, racts, icd, acts, out, nn, rinfo, qw, l, i); break;
        case 2: apiqv_run<2, BLACK>(slab, seed, htab, racts, icd, acts, out, nn, rinfo, qw, l, i); break;
        default: apiqv_run<3, BLACK>(slab, seed, htab, racts, icd, acts, out, nn, rinfo, qw, l, i); break;
    }
}

// ----------------------------------------------------------------------------- API step, paired, random opponent
// k_env_step_api<true> (the random opponent answers inside the step: env_step_vs,
// chess_v2.py:219-294 with opponent_policy set) on the paired driver.  Half A: the agent's
// validated action with set-wise generation (W0 picks the opponent's reply in move-set
// order, draw d); half B: the reply -- or, for a board whose state stays or whose episode
// ended with the agent's move, its own moves again -- with the per-piece generation the
// mask needs; for a BLACK agent, half C (run only when some board of the workgroup resets):
// the opponent's opening from the reset position (move-set order table, the next draw).  A
// WHITE agent's reset board takes the start position's cached moves.  The agent's pick (the
// next draw, action order) and the outputs as in k_env_step_api2.  Same draws in the same
// order as the one-wave kernel.
template <bool BLACK>
__global__ void __launch_bounds__(2 * PAIR_BOARDS * PAIRS_WG) PAIR_ATTR
    k_env_step_api2_vs(uint8_t* __restrict__ slab, uint64_t seed, u64* __restrict__ htab,
                       const uint16_t* __restrict__ racts, const EnvDev::InitCache* __restrict__ icd,
                       const uint16_t* __restrict__ acts, const ApiOut* __restrict__ outp, int nn,
                       u32 rinfo /* autoreset << 17 | ic.table << 16 | ic.total */) {
    constexpr int OPP = BLACK ? 2 : 1;
    constexpr bool API = true;
    constexpr int blk0 = 0;
    const int autoreset = (rinfo >> 17) & 1;
    rinfo &= 0x1FFFFu;
    ApiOut out;
    PAIR_PROLOGUE_ACT(acts, out = *outp; asm volatile("" : "+s"(out.rw), "+s"(out.dn), "+s"(out.rs), "+s"(out.mask),
                                                                  "+s"(out.obs), "+s"(out.cnt), "+s"(out.pick), "+s"(out.ms));)
    PairScratch scr{&L.slots[0][l]};
    const uint16_t* const sw_tab = C.racts + RESET_ACTS_MAX;  // the start position's picks in move-set order
    const bool done0 = (s.meta & M_DONE) != 0;              // chess_v2.py:245-251
    const bool cap = mc_of(s.meta) > MOVES_MAX;             // 252-258
    const bool white = (s.meta & M_WHITE) != 0;             // the agent's colour
    const bool pre = live && !done0 && !cap;
    bool valid = false;
    if (role == 0) {  // chess_v2.py:240-242, on the pre-move board
        valid = quick_legal(s, a);
        L.act[l] = valid ? 1u : 0u;
        L.draw[l] = (pre && valid) ? 1u : 0u;  // W1 reads it in phase 1 (MV_LDS)
    }
    u32 x0 = 0, x1 = 0, x2 = 0;
    PairHalf H;
    // ---- half A: the agent's move; the opponent's position generated set-wise
    pair_half<false, false, true, true>(
        L, role, l, role == 0 ? (pre && valid) : pre, false, s, a, nullptr, L.draw, h, H,
        [&] {
            x0 = philox_x0(C.seed, (u32)i, d);
            x1 = philox_x0(C.seed, (u32)i, d + 1);
            x2 = philox_x0(C.seed, (u32)i, d + 2);
            L.x0[l] = x0;
            L.x1[l] = x1;
            L.x2[l] = x2;
        },
        PairNoop{});
    if (role) valid = L.act[l] != 0;
    else {
        x0 = L.x0[l];
        x1 = L.x1[l];
        x2 = L.x2[l];
    }
    StepOut o = {0, 0, R_NONE, 0};
    bool cont = false;  // the opponent replies
    if (!valid) {
        o.reward = -10;
        o.done = done0 ? 1 : 0;
        o.reason = R_INVALID;
    } else if (done0) {
        o.done = 1;
        o.reason = R_DONE_ALREADY;
    } else if (cap) {
        o.done = 1;
        o.reason = R_MOVE_CAP;
    } else if (H.both) {
        o.done = 1;
        o.reason = R_BOTH_CHECKED;
    } else {
        s = pair_settle(H, white);
        o.reward = -10 + H.mr;  // Q9
        o.moved = 1;
        if (H.c >= 3) { o.done = 1; o.reason = R_REPETITION; }
        if (H.c == 0) { o.done = 1; o.reason = R_WINDOW_FULL; }
        if (H.ms.total == 0 && H.opp_chk) {  // 270-272
            s.meta |= M_DONE;
            o.done = 1;
            o.reward += 100;
            o.reason = R_MATE;
        }
        if (!o.done && H.ms.total == 0) {  // 120-122: the opponent's policy "resigns"
            s.meta |= M_DONE;
            o.done = 1;
            o.reason = R_OPP_NO_MOVE;
        }
        cont = !o.done;
    }
    int nd = cont ? 1 : 0;  // draws taken so far
    int oa = A_NONE;
    if (role == 0) {
        if (cont) oa = sw_pick_lds(L, l, H.g, H.cw, H.ms.total, (int)scale_rank(x0, (u32)H.ms.total));
        L.oa[l] = (u32)oa;
    } else if (live) {
        h.commit();  // the agent ply's window write lands before the reply probes the table
    }
    // ---- half B: the reply, or the board's own moves again (per-piece, for the mask)
    const Pos s1 = s;
    pair_half<false, true>(L, role, l, cont, live && !cont, s1, oa, L.oa, nullptr, h, H, PairNoop{}, PairNoop{});
    bool alone = false;  // the state stays but no moves were generated for it
    if (cont) {
        if (H.both) {  // the reply left both kings checked: the engine raises, the env ends
            o.reason = R_BOTH_CHECKED;
            o.done = 1;
            alone = true;
        } else {
            s = pair_settle(H, !white);
            o.reward -= H.mr;  // 283
            if (H.c >= 3) { o.done = 1; o.reason = R_REPETITION; }
            if (H.c == 0) { o.done = 1; o.reason = R_WINDOW_FULL; }
            if (H.ms.total == 0 && H.opp_chk) {  // 285-288
                s.meta |= M_DONE;
                o.done = 1;
                o.reward -= 100;
                o.reason = R_MATED;
            }
            if (s.meta & M_WHITE) s.meta += (1u << M_MC_SHIFT);  // 291-292
        }
    }
    nst += 1;
    const bool reset = live && autoreset && o.done;
    if (reset) {  // chess_v2.py:183-206
        s = rp;
        h.bump_gen();
        alone = false;
    }
    if constexpr (BLACK) {
        // ---- half C: the opponent's opening after a reset (208-216), when some board of the
        // workgroup needs it; the other boards keep half B's generation
        const unsigned long long vote = __ballot(reset);
        if (l == 0) L.vote[role] = vote != 0 ? 1u : 0u;
        if (role && live) h.commit();
        pair_barrier();
        bool any = false;
#pragma unroll
        for (int q = 0; q < PAIRS_WG; q++) any = any || Ls[q].vote[0] != 0 || Ls[q].vote[1] != 0;
        if (any) {
            const Gen gB = H.g;
            const MoveSet msB = H.ms;
            const u32 xo = nd ? x1 : x0;
            const int op = (int)sw_tab[scale_rank(xo, C.rtotal)];
            if (role == 0) L.oa[l] = (u32)op;
            const Pos s0 = s;
            pair_half<false, true>(L, role, l, reset, false, s0, op, L.oa, nullptr, h, H, PairNoop{}, PairNoop{});
            if (reset) {
                s = pair_settle(H, true);
                s.meta = (s.meta & ~(u32)M_DONE) + (1u << M_MC_SHIFT);
                nd += 1;
            } else {
                H.g = gB;
                H.ms = msB;
            }
        }
    }
    // W0: every own piece's targets into its slot (fast pawns from their origin sets; a WHITE
    // agent's reset board from the start position's cache); castles and the enemy map to W1
    const bool cached = reset && !BLACK;
    if (role == 0) {
        if (cached) {
#pragma unroll
            for (int j = 0; j < SCRATCH_SLOTS; j++) scr.put(j, C.icd->slots[j]);
        } else if (!H.ms.big) {
            for (u64 fp = H.ms.fastp; fp; fp &= fp - 1) {
                const int sq = ctz(fp);
                scr.put(ordinal(H.g.own, sq), fast_pawn_targets(H.ms, sq, H.g.white));
            }
        }
        L.nmeta[l] = H.g.castles;
        L.enemy[l] = H.g.enemy_att;
    }
    pair_barrier();
    Gen g = H.g;
    MoveSet ms = H.ms;
    if (role) {
        g.castles = L.nmeta[l];
        g.enemy_att = L.enemy[l];
    }
    if (cached) ic_moves(*C.icd, g, ms);
    if (alone && live) {  // the big-board path: legal targets per piece, no slots
        gen_init(s, g);
        moveset_clear(ms);
        ms.big = true;
        ms.total = count_legal(s, g);
    }
    if (out.mask && live) {
        u64* om = out.mask + i;
        const size_t N = out.ms;
        if (!ms.big) {  // W1 squares 0..31, W0 32..63 and the castles word
            const int q0 = role ? 0 : 32;
            int j = popc(g.own & below(q0));
#pragma unroll 8
            for (int sq = q0; sq < q0 + 32; sq++) {
                const bool b = (g.own >> sq) & 1;
                const u64 v = scr.get(j & (SCRATCH_SLOTS - 1));
                om[sq * N] = b ? v : 0ull;
                j += b ? 1 : 0;
            }
            if (role == 0) {
                u64 c = 0;
                if (g.castles & 1) c |= g.white ? (1ull << 1) : (1ull << 3);
                if (g.castles & 2) c |= g.white ? (1ull << 0) : (1ull << 2);
                om[64 * N] = c;
            }
        } else if (role) {
            write_mask(s, g, ms, scr, om, N);
        }
    }
    const PairIO io = store_io(slab, nn);
    if (role == 0) {
        if (live) {
            const u32 xp = nd == 0 ? x0 : nd == 1 ? x1 : x2;
            uint16_t p = (uint16_t)A_NONE;
            u32 dn = d + (u32)nd;
            if (out.pick) {
                if (cached && C.rtable) {
                    p = C.racts[scale_rank(xp, C.rtotal)];
                } else if (ms.total > 0) {
                    p = (uint16_t)select_action_swar(s, g, ms, scr, (int)scale_rank(xp, (u32)ms.total));
                }
                dn += ms.total > 0 ? 1u : 0u;
                out.pick[i] = p;
                io.act[i] = p;
            }
            io.draw[i] = dn;
        }
    } else if (live) {
        if (out.obs) write_obs(s, out.obs + 64 * (size_t)i);
        if (out.cnt) out.cnt[i] = ms.total;
        out.rw[i] = o.reward;
        out.dn[i] = (uint8_t)o.done;
        out.rs[i] = (uint8_t)o.reason;
        h.commit();
        io.store(i, s);
        h.flush(g0);
        io.nsteps[i] = nst;
        io.reward[i] = o.reward;
        io.done[i] = (uint8_t)o.done;
        io.reason[i] = (uint8_t)o.reason;
    }
}

__global__ void __launch_bounds__(BLOCK) k_select(EnvDev e) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= e.n) return;
    Pos s = e.st.load(i);
    PolicyCtx pc = {e.seed, (u32)i, e.draw[i]};
    e.act[i] = (uint16_t)selfplay_pick(s, pc);
    e.draw[i] = pc.draw;
}

#include "gc_fide_kernels.h"

// The API step under the optional FIDE rules (gc_fide.h; VERDICT r03 missing #3), one lane per
// board as the mode's other kernels: the external action validated and played by
// gcf::fenv_step (en passant, promotion to a queen, FIDE castling), auto-reset to the start
// position, then k_env_step_api's outputs from the new position's legal targets per own
// square (the action-id order of the mask and of the pick; castles in word 64).
template <bool OPP>
__global__ void __launch_bounds__(BLOCK) k_fenv_step_api(EnvDev e, const uint16_t* __restrict__ acts,
                                                         int32_t* __restrict__ rw, uint8_t* __restrict__ dn,
                                                         uint8_t* __restrict__ rs, u64* __restrict__ mask,
                                                         int8_t* __restrict__ obs, int32_t* __restrict__ cnt,
                                                         uint16_t* __restrict__ pick_out, int autoreset, size_t mstride) {
    LDS_SCRATCH_DECL;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= e.n) return;
    Pos s = e.st.load(i);
    u32 g0 = e.hgen[i], d = e.draw[i], nst = e.nsteps[i];
    DevHist h = e.hist(i, g0);
    gcf::FGen f;
    const StepOut o = OPP ? gcf::fenv_step_vs<true>(s, h, (int)acts[i], f, scr, e.seed, (u32)i, d)
                          : gcf::fenv_step<true>(s, h, (int)acts[i], f);
    bool have = o.moved;
    nst += 1;
    if (autoreset && o.done) {  // a BLACK agent's opponent opens (chess_v2.py:208-216)
        s = fide_reset_pos(e);
        h.bump_gen();
        gcf::fgen(s, f);
        if (OPP && e.agent_black) {
            h.commit();
            gcf::fenv_open_vs(s, h, f, scr, e.seed, (u32)i, d);
        }
        have = true;
    }
    if (!have) gcf::fgen(s, f);
    const size_t N = mstride;
    u64 cw = 0;  // bit c = action 4096 + c
    if (f.g.castles & 1) cw |= f.g.white ? (1ull << 1) : (1ull << 3);
    if (f.g.castles & 2) cw |= f.g.white ? (1ull << 0) : (1ull << 2);
    int total = popc(cw);
    for (int sq = 0; sq < 64; sq++) {
        const u64 tg = ((f.g.own >> sq) & 1) ? gcf::ftargets(s, f, sq, type_at(s, sq)) : 0ull;
        if (mask) mask[sq * N + i] = tg;
        total += popc(tg);
    }
    if (mask) mask[64 * N + i] = cw;
    rw[i] = o.reward;
    dn[i] = (uint8_t)o.done;
    rs[i] = (uint8_t)o.reason;
    if (cnt) cnt[i] = total;
    if (obs) write_obs(s, obs + 64 * (size_t)i);
    if (pick_out) {  // the k-th legal action in action-id order (as pick_mask_order)
        uint16_t p = (uint16_t)A_NONE;
        if (total > 0) {
            int k = (int)policy_index(e.seed, (u32)i, d++, (u32)total);
            u64 pcs = f.g.own;
            while (pcs && p == (uint16_t)A_NONE) {
                const int sq = ctz(pcs);
                pcs &= pcs - 1;
                u64 tg = gcf::ftargets(s, f, sq, type_at(s, sq));
                const int c = popc(tg);
                if (k < c) {
                    for (; k > 0; k--) tg &= tg - 1;
                    p = (uint16_t)(sq * 64 + ctz(tg));
                } else {
                    k -= c;
                }
            }
            for (int c = 0; c < 4 && p == (uint16_t)A_NONE; c++) {
                if (!((cw >> c) & 1)) continue;
                if (k == 0) p = (uint16_t)(4096 + c);
                else k--;
            }
        }
        pick_out[i] = p;
        e.act[i] = p;
    }
    h.commit();
    e.st.store(i, s);
    h.flush(g0);
    e.draw[i] = d;
    e.nsteps[i] = nst;
    e.reward[i] = o.reward;
    e.done[i] = (uint8_t)o.done;
    e.reason[i] = (uint8_t)o.reason;
}


// ----------------------------------------------------------------------------- host side
static inline int grid_for(int n) { return (n + BLOCK - 1) / BLOCK; }

template <class T>
static int dalloc(T** p, size_t count) {
    if (count == 0) count = 1;
    hipError_t e = hipMalloc((void**)p, count * sizeof(T));
    if (e != hipSuccess) return fail(std::string("hipMalloc: ") + hipGetErrorString(e));
    return 0;
}

struct gc_engine {
    int device = 0;
    hipStream_t stream = nullptr;
    int cap_n = 0, cap_list = 0;
    u64* bb = nullptr; u32* meta = nullptr;       // input states
    u64* bb2 = nullptr; u32* meta2 = nullptr;     // output states
    // The host-facing buffers of one call are views into ONE device block (dio), laid out for
    // the call's n by engine_layout, mirrored by a pinned host block (hio): a call stages its
    // inputs with one host-to-device copy and returns its outputs with one copy back (a
    // single-board call is latency-bound: every copy is a round trip)
    uint8_t* dio = nullptr; uint8_t* hio = nullptr; size_t io_cap = 0;
    int8_t* mbox = nullptr; uint8_t* m8 = nullptr; uint8_t* side = nullptr;
    uint16_t* acts = nullptr; int32_t* i32a = nullptr; int32_t* i32b = nullptr;
    uint16_t* list = nullptr; uint64_t* u64o = nullptr;
    int rules = 0;  // 0 reference (lib.rs), 1 FIDE (gc_fide.h)
    // small calls (a layout within ENGINE_ZC_BYTES) stage in host-mapped coherent memory that
    // the kernels read and write directly: one launch and no copy per call, where the
    // staged form paid a copy each way (two more dispatches) around it
    uint8_t* zc = nullptr; uint8_t* zcd = nullptr; bool zc_on = false;
    // one-position calls under the reference rules go to the engine server (k_engine_server)
    struct EngBox* srv = nullptr; struct EngBox* srv_d = nullptr;
    hipStream_t srv_stream = nullptr;
    uint32_t srv_seq = 0, srv_launch = 0, srv_next_launch = 0;
    // one call at a time per engine: ctypes releases the GIL, and a call's staging buffers
    // and the server's mailbox are the engine's own
    std::mutex mu;
};
#define ENGINE_ZC_BYTES 65536
// byte offsets of the views for n boards and a list capacity lc (256-B aligned)
struct EngineLayout {
    size_t mbox, m8, side, acts, i32a, i32b, list, end;
};
static EngineLayout engine_offsets(size_t n, size_t lc) {
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    EngineLayout o;
    o.mbox = 0;
    o.m8 = up(o.mbox + 64 * n);
    o.side = up(o.m8 + 8 * n);
    o.acts = up(o.side + n);
    o.i32a = up(o.acts + 2 * n);
    o.i32b = up(o.i32a + 4 * n);
    o.list = up(o.i32b + 4 * n);
    o.end = up(o.list + 2 * lc * n);
    return o;
}
static EngineLayout engine_layout(gc_engine* e, int n, int lc, uint8_t* base) {
    EngineLayout o = engine_offsets((size_t)n, (size_t)lc);
    e->mbox = reinterpret_cast<int8_t*>(base + o.mbox);
    e->m8 = base + o.m8;
    e->side = base + o.side;
    e->acts = reinterpret_cast<uint16_t*>(base + o.acts);
    e->i32a = reinterpret_cast<int32_t*>(base + o.i32a);
    e->i32b = reinterpret_cast<int32_t*>(base + o.i32b);
    e->list = reinterpret_cast<uint16_t*>(base + o.list);
    return o;
}
static bool engine_zc_enabled() {
    static const bool off = getenv("GC_ENGINE_ZC") && atoi(getenv("GC_ENGINE_ZC")) == 0;  // A/B
    return !off;
}

static void engine_free_bufs(gc_engine* e) {
    void* ps[] = {e->bb, e->meta, e->bb2, e->meta2, e->dio, e->u64o};
    for (void* p : ps) if (p) (void)hipFree(p);
    if (e->hio) (void)hipHostFree(e->hio);
    if (e->zc) (void)hipHostFree(e->zc);
    e->zc = nullptr; e->zcd = nullptr; e->zc_on = false;
    e->bb = nullptr; e->meta = nullptr; e->bb2 = nullptr; e->meta2 = nullptr; e->dio = nullptr; e->hio = nullptr;
    e->mbox = nullptr; e->m8 = nullptr; e->side = nullptr; e->acts = nullptr; e->i32a = nullptr; e->i32b = nullptr;
    e->list = nullptr; e->u64o = nullptr;
    e->cap_n = 0; e->cap_list = 0; e->io_cap = 0;
}

static int engine_reserve(gc_engine* e, int n, int listcap) {
    if (n <= e->cap_n && listcap <= e->cap_list) return 0;
    int nn = n > e->cap_n ? n : e->cap_n, lc = listcap > e->cap_list ? listcap : e->cap_list;
    engine_free_bufs(e);
    const size_t io = engine_offsets((size_t)nn, (size_t)lc).end;
    if (dalloc(&e->bb, (size_t)NBB * nn) || dalloc(&e->meta, nn) || dalloc(&e->bb2, (size_t)NBB * nn) ||
        dalloc(&e->meta2, nn) || dalloc(&e->dio, io) || dalloc(&e->u64o, nn))
        return -1;
    hipError_t he = hipHostMalloc((void**)&e->hio, io, hipHostMallocDefault);
    if (he != hipSuccess) return fail(std::string("hipHostMalloc: ") + hipGetErrorString(he));
    e->io_cap = io;
    e->cap_n = nn;
    e->cap_list = lc;
    return 0;
}
// one call's staging: the inputs present (side / acts may be null) into the pinned block, one
// copy to the device; the views laid out for (n, lc)
static int engine_stage(gc_engine* e, int n, int lc, const int8_t* boards, const uint8_t* meta, const uint8_t* side,
                        const uint16_t* acts, EngineLayout& o) {
    e->zc_on = engine_zc_enabled() && engine_offsets((size_t)n, (size_t)lc).end <= ENGINE_ZC_BYTES;
    if (e->zc_on && !e->zc) {
        HIPCHK(hipHostMalloc((void**)&e->zc, ENGINE_ZC_BYTES, hipHostMallocMapped | hipHostMallocCoherent));
        HIPCHK(hipHostGetDevicePointer((void**)&e->zcd, e->zc, 0));
    }
    uint8_t* h = e->zc_on ? e->zc : e->hio;
    o = engine_layout(e, n, lc, e->zc_on ? e->zcd : e->dio);
    std::memcpy(h + o.mbox, boards, (size_t)64 * n);
    std::memcpy(h + o.m8, meta, (size_t)8 * n);
    size_t end = o.m8 + (size_t)8 * n;
    if (side) { std::memcpy(h + o.side, side, (size_t)n); end = o.side + n; }
    if (acts) { std::memcpy(h + o.acts, acts, (size_t)2 * n); end = o.acts + (size_t)2 * n; }
    if (!e->zc_on) HIPCHK(hipMemcpyAsync(e->dio, e->hio, end, hipMemcpyHostToDevice, e->stream));
    return 0;
}
// the byte range [a, b) of the device block back into the pinned one, then wait (a small
// call's outputs are already in host memory: only the wait, and the range into hio)
static int engine_fetch(gc_engine* e, size_t a, size_t b) {
    if (!e->zc_on) HIPCHK(hipMemcpyAsync(e->hio + a, e->dio + a, b - a, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    if (e->zc_on) std::memcpy(e->hio + a, e->zc + a, b - a);
    return 0;
}

static int check_boards(int n, const int8_t* boards) {
    for (size_t k = 0; k < (size_t)64 * n; k++)
        if (boards[k] < -6 || boards[k] > 6) return fail("piece id out of range [-6, 6] at index " + std::to_string(k));
    return 0;
}

// side: staged when given, and the side to move of the import unless side_import is false
static int engine_upload(gc_engine* e, int n, const int8_t* boards, const uint8_t* meta, const uint8_t* side,
                         EngineLayout& o, int lc = 1, const uint16_t* acts = nullptr, bool side_import = true) {
    if (n <= 0) return fail("n must be > 0");
    if (!boards || !meta) return fail("null boards/meta");
    if (check_boards(n, boards)) return -1;
    HIPCHK(hipSetDevice(e->device));
    if (engine_stage(e, n, lc, boards, meta, side, acts, o)) return -1;
    if (!side_import) side = nullptr;
    SoA st{e->bb, e->meta, n};
    if (e->rules) k_fimport<<<grid_for(n), BLOCK, 0, e->stream>>>(e->mbox, e->m8, side ? e->side : nullptr, st);
    else k_import<<<grid_for(n), BLOCK, 0, e->stream>>>(e->mbox, e->m8, side ? e->side : nullptr, st);
    HIPCHK(hipGetLastError());
    return 0;
}

static void engine_export(gc_engine* e, SoA st) {
    if (e->rules) k_fexport<<<grid_for(st.n), BLOCK, 0, e->stream>>>(st, e->mbox, e->m8);
    else k_export<<<grid_for(st.n), BLOCK, 0, e->stream>>>(st, e->mbox, e->m8);
}

// rules 0: the reference's (default); 1: FIDE (gc_fide.h; meta8[7] = en-passant file + 1)
extern "C" int gc_engine_set_rules(gc_engine* e, int rules) {
    if (!e) return fail("null engine");
    std::lock_guard<std::mutex> lk(e->mu);
    if (rules != 0 && rules != 1) return fail("rules must be 0 (reference) or 1 (fide)");
    e->rules = rules;
    return 0;
}

extern "C" int gc_engine_create(int device, gc_engine** out) {
    if (!out) return fail("null out pointer");
    int nd = 0;
    HIPCHK(hipGetDeviceCount(&nd));
    if (device < 0 || device >= nd) return fail("device index out of range");
    gc_engine* e = new gc_engine();
    e->device = device;
    HIPCHK(hipSetDevice(device));
    HIPCHK(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
    if (engine_reserve(e, 256, 256)) { delete e; return -1; }
    *out = e;
    return 0;
}

// ---- resident servers at process exit: a server wave exits after SRV_IDLE_MS without a
// request, so a process that ends right after its last call (without destroying the env or
// engine) could end with the wave still resident.  Every running server is registered here;
// an atexit handler asks each to QUIT through its host-mapped mailbox and waits (host memory
// only, no HIP call: the runtime may be tearing down) until it has marked its exit.
struct SrvReg {
    u32 *req_seq, *op, *exited;      // the mailbox (host-mapped)
    const u32 *seq, *launch;         // the owner's last served sequence number and launch id
};
static std::mutex g_srvreg_mu;
static std::vector<std::pair<const void*, SrvReg>> g_srvreg;
static void srv_quit_all() {
    std::lock_guard<std::mutex> lk(g_srvreg_mu);
    const bool log = getenv("GC_SRV_EXIT_LOG") != nullptr;  // (tests: which servers this stopped)
    for (auto& it : g_srvreg) {
        const SrvReg& r = it.second;
        if (!*r.launch || __atomic_load_n(r.exited, __ATOMIC_ACQUIRE) == *r.launch) continue;
        __atomic_store_n(r.op, (u32)SRV_QUIT, __ATOMIC_RELAXED);
        __atomic_store_n(r.req_seq, *r.seq + 1, __ATOMIC_RELEASE);
        const auto t0 = std::chrono::steady_clock::now();
        while (__atomic_load_n(r.exited, __ATOMIC_ACQUIRE) != *r.launch &&
               std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(2 * SRV_IDLE_MS)) {
        }
        if (log)
            fprintf(stderr, "gymchess: server of %p %s at exit\n", it.first,
                    __atomic_load_n(r.exited, __ATOMIC_ACQUIRE) == *r.launch ? "stopped" : "did not answer");
    }
    g_srvreg.clear();
}
static void srv_register(const void* owner, const SrvReg& r) {
    std::lock_guard<std::mutex> lk(g_srvreg_mu);
    static bool hooked = false;
    if (!hooked) {
        std::atexit(srv_quit_all);
        hooked = true;
    }
    for (auto& it : g_srvreg)
        if (it.first == owner) return;
    g_srvreg.emplace_back(owner, r);
}
static void srv_unregister(const void* owner) {
    std::lock_guard<std::mutex> lk(g_srvreg_mu);
    for (size_t k = 0; k < g_srvreg.size(); k++)
        if (g_srvreg[k].first == owner) {
            g_srvreg.erase(g_srvreg.begin() + (long)k);
            return;
        }
}

// ---- one resident server per device.  A resident wave holds its hardware
// queue until it exits, and HIP maps a process's streams onto GPU_MAX_HW_QUEUES (4 on the box)
// queues: with more streams than that, work on a stream that shares a queue with a resident
// server waits behind it until it idles out (SRV_IDLE_MS) -- ~50 ms per call for single-board
// envs stepped round-robin, or env.step mixed with ChessEngine calls.  So at most one server
// runs per device: a request to another owner's server, and every launch of this library on
// the device (SRV_QUIESCE, devsrv_quiesce), first stops the resident one (QUIT, its stream
// drained).  The slot's mutex is held for a whole server call (lock order: an engine's own
// mutex, then the slot's), so a server's state is only touched under it.
#define GC_MAX_DEVICES 64
struct DevSrv {
    std::recursive_mutex mu;
    std::atomic<void*> owner{nullptr};  // the env / engine whose server may be resident
    int (*stop)(void*) = nullptr;       // its stop (QUIT + drain)
};
static DevSrv g_devsrv[GC_MAX_DEVICES];
static DevSrv& devsrv(int dev) { return g_devsrv[(unsigned)dev % GC_MAX_DEVICES]; }
// (held: s.mu)
static int devsrv_stop_locked(DevSrv& s) {
    void* o = s.owner.exchange(nullptr, std::memory_order_acq_rel);
    return o ? s.stop(o) : 0;
}
// (Lock-free when no server is resident.  Callers on other threads may claim the slot between
// this check and their own launch: that launch then queues behind the new server until the
// server stops -- at the next call of another owner, or by itself after SRV_IDLE_MS without a
// request -- a delay, never a wrong result.)
static int devsrv_quiesce(int dev) {
    DevSrv& s = devsrv(dev);
    if (!s.owner.load(std::memory_order_acquire)) return 0;
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    return devsrv_stop_locked(s);
}
// (held: s.mu) the slot for `owner`: another owner's server is stopped first
static int devsrv_claim(DevSrv& s, void* owner, int (*stop)(void*)) {
    void* o = s.owner.load(std::memory_order_acquire);
    if (o && o != owner && devsrv_stop_locked(s)) return -1;
    s.stop = stop;
    s.owner.store(owner, std::memory_order_release);
    return 0;
}
static void devsrv_release(DevSrv& s, void* owner) {
    void* o = owner;
    s.owner.compare_exchange_strong(o, nullptr, std::memory_order_acq_rel);
}

// ---- the engine server's host side (the single-board server's protocol, srv_call)
static bool eng_srv_enabled() {
    static const bool off = getenv("GC_ENGINE_SERVER") && atoi(getenv("GC_ENGINE_SERVER")) == 0;  // A/B
    return !off;
}
static int eng_srv_stop(gc_engine* e) {
    DevSrv& s = devsrv(e->device);
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    devsrv_release(s, e);
    if (!e->srv_launch) return 0;
    EngBox* b = e->srv;
    __atomic_store_n(&b->op, (u32)SRV_QUIT, __ATOMIC_RELAXED);
    __atomic_store_n(&b->req_seq, e->srv_seq + 1, __ATOMIC_RELEASE);  // (never served: QUIT)
    const hipError_t he = hipStreamSynchronize(e->srv_stream);
    __atomic_store_n(&b->req_seq, e->srv_seq, __ATOMIC_RELEASE);
    e->srv_launch = 0;
    if (he != hipSuccess) return fail(std::string("engine server: ") + hipGetErrorString(he));
    return 0;
}
// one op on one position; the response lands in e->srv
static int eng_srv_stop_v(void* e) { return eng_srv_stop(static_cast<gc_engine*>(e)); }
static int eng_srv_call(gc_engine* e, int op, const int8_t* board, const uint8_t* meta, bool white, int arg) {
    HIPCHK(hipSetDevice(e->device));
    DevSrv& s = devsrv(e->device);
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    if (devsrv_claim(s, e, eng_srv_stop_v)) return -1;
    if (!e->srv) {
        HIPCHK(hipHostMalloc((void**)&e->srv, sizeof(EngBox), hipHostMallocMapped | hipHostMallocCoherent));
        memset(e->srv, 0, sizeof(EngBox));
        HIPCHK(hipHostGetDevicePointer((void**)&e->srv_d, e->srv, 0));
        HIPCHK(hipStreamCreateWithFlags(&e->srv_stream, hipStreamNonBlocking));
    }
    EngBox* b = e->srv;
    const u32 seq = e->srv_seq + 1;
    memcpy(b->board, board, 64);
    memcpy(b->meta, meta, 8);
    __atomic_store_n(&b->op, (u32)op, __ATOMIC_RELAXED);
    __atomic_store_n(&b->white, white ? 1u : 0u, __ATOMIC_RELAXED);
    __atomic_store_n(&b->arg, (u32)arg, __ATOMIC_RELAXED);
    __atomic_store_n(&b->req_seq, seq, __ATOMIC_RELEASE);  // last
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned k = 0;; k++) {
        if (!e->srv_launch || __atomic_load_n(&b->exited, __ATOMIC_ACQUIRE) == e->srv_launch) {
            if (e->srv_launch) HIPCHK(hipStreamSynchronize(e->srv_stream));  // drained (idle exit)
            e->srv_launch = ++e->srv_next_launch;
            srv_register(e, SrvReg{&b->req_seq, &b->op, &b->exited, &e->srv_seq, &e->srv_launch});
            k_engine_server<<<1, 64, 0, e->srv_stream>>>(e->srv_d, e->srv_seq, e->srv_launch);
            HIPCHK(hipGetLastError());
        }
        if (__atomic_load_n(&b->resp_seq, __ATOMIC_ACQUIRE) == seq) break;
        if ((k & 1023) == 1023) {
            const hipError_t q = hipStreamQuery(e->srv_stream);
            if (q != hipSuccess && q != hipErrorNotReady) return fail(std::string("engine server: ") + hipGetErrorString(q));
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10)) {
                (void)eng_srv_stop(e);
                return fail("engine server: no answer within 10 s");
            }
        }
    }
    e->srv_seq = seq;
    return 0;
}
static bool eng_srv_use(const gc_engine* e, int n) { return n == 1 && !e->rules && eng_srv_enabled(); }

extern "C" int gc_engine_destroy(gc_engine* e) {
    if (!e) return 0;
    (void)hipSetDevice(e->device);
    (void)eng_srv_stop(e);
    srv_unregister(e);
    if (e->srv_stream) (void)hipStreamDestroy(e->srv_stream);
    if (e->srv) (void)hipHostFree(e->srv);
    (void)hipStreamSynchronize(e->stream);
    engine_free_bufs(e);
    (void)hipStreamDestroy(e->stream);
    delete e;
    return 0;
}

extern "C" int gc_engine_get_possible_moves(gc_engine* e, int n, const int8_t* boards, const uint8_t* meta,
                                            const uint8_t* player_white, int attack, uint16_t* moves, int cap,
                                            int32_t* counts) {
    if (!e || !moves || !counts || !player_white) return fail("null argument");
    std::lock_guard<std::mutex> lk(e->mu);
    if (cap <= 0) return fail("cap must be > 0");
    if (eng_srv_use(e, n) && cap <= ENG_SRV_CAP) {
        if (!boards || !meta) return fail("null boards/meta");
        if (check_boards(1, boards)) return -1;
        if (eng_srv_call(e, ENG_LIST, boards, meta, player_white[0] != 0, attack ? 1 : 0)) return -1;
        const int c = (int)e->srv->count;
        memcpy(moves, e->srv->moves, (size_t)2 * (c < cap ? c : cap));
        counts[0] = c;
        return 0;
    }
    if (devsrv_quiesce(e->device) || engine_reserve(e, n, cap)) return -1;
    EngineLayout o;
    if (e->rules) {
        if (engine_upload(e, n, boards, meta, player_white, o, cap)) return -1;
        k_flist<<<grid_for(n), BLOCK, 0, e->stream>>>(SoA{e->bb, e->meta, n}, attack ? 1 : 0, cap, e->list, e->i32a);
    } else {  // one launch: import + list
        if (n <= 0) return fail("n must be > 0");
        if (!boards || !meta) return fail("null boards/meta");
        if (check_boards(n, boards)) return -1;
        HIPCHK(hipSetDevice(e->device));
        if (engine_stage(e, n, cap, boards, meta, player_white, nullptr, o)) return -1;
        k_list_mb<<<grid_for(n), BLOCK, 0, e->stream>>>(e->mbox, e->m8, e->side, n, attack ? 1 : 0, cap, e->list, e->i32a);
    }
    HIPCHK(hipGetLastError());
    if (engine_fetch(e, o.i32a, o.list + (size_t)2 * cap * n)) return -1;
    std::memcpy(moves, e->hio + o.list, (size_t)2 * cap * n);
    std::memcpy(counts, e->hio + o.i32a, (size_t)4 * n);
    return 0;
}

extern "C" int gc_engine_get_castle_moves(gc_engine* e, int n, const int8_t* boards, const uint8_t* meta,
                                          const uint8_t* player_white, uint16_t* moves, int32_t* counts) {
    if (!e || !moves || !counts || !player_white) return fail("null argument");
    std::lock_guard<std::mutex> lk(e->mu);
    if (eng_srv_use(e, n)) {
        if (!boards || !meta) return fail("null boards/meta");
        if (check_boards(1, boards)) return -1;
        if (eng_srv_call(e, ENG_CASTLE, boards, meta, player_white[0] != 0, 0)) return -1;
        const u32 c = e->srv->count;
        int k = 0;  // reference order (QS then KS, lib.rs:992,1011)
        if (c & 2u) moves[k++] = A_QSW;
        if (c & 1u) moves[k++] = A_KSW;
        if (c & 8u) moves[k++] = A_QSB;
        if (c & 4u) moves[k++] = A_KSB;
        counts[0] = k;
        return 0;
    }
    if (devsrv_quiesce(e->device) || engine_reserve(e, n, 2)) return -1;
    EngineLayout o;
    if (engine_upload(e, n, boards, meta, player_white, o, 2)) return -1;
    std::vector<u64> mask(e->rules ? (size_t)65 * n : 0);
    if (e->rules) {
        u64* dmask = nullptr;
        if (dalloc(&dmask, (size_t)65 * n)) return -1;
        k_fmask<<<grid_for(n), BLOCK, 0, e->stream>>>(SoA{e->bb, e->meta, n}, dmask, nullptr);
        hipError_t le = hipGetLastError();
        hipError_t ce = hipMemcpyAsync(mask.data(), dmask, (size_t)8 * 65 * n, hipMemcpyDeviceToHost, e->stream);
        hipError_t se = hipStreamSynchronize(e->stream);
        (void)hipFree(dmask);
        if (le != hipSuccess || ce != hipSuccess || se != hipSuccess) return fail("castle mask kernel failed");
    } else {  // the castle word per board into the layout's int32 row
        k_castle_word<<<grid_for(n), BLOCK, 0, e->stream>>>(SoA{e->bb, e->meta, n}, e->i32a);
        HIPCHK(hipGetLastError());
        if (engine_fetch(e, o.i32a, o.i32a + (size_t)4 * n)) return -1;
    }
    for (int i = 0; i < n; i++) {  // unpack in reference order (QS then KS, lib.rs:992,1011)
        const u64 c = e->rules ? mask[(size_t)65 * i + 64] : (u64)reinterpret_cast<const int32_t*>(e->hio + o.i32a)[i];
        int k = 0;
        uint16_t* o = moves + 2 * (size_t)i;
        if (c & (1ull << 1)) o[k++] = A_QSW;
        if (c & (1ull << 0)) o[k++] = A_KSW;
        if (c & (1ull << 3)) o[k++] = A_QSB;
        if (c & (1ull << 2)) o[k++] = A_KSB;
        counts[i] = k;
    }
    return 0;
}

extern "C" int gc_engine_next_state(gc_engine* e, int n, const int8_t* boards, const uint8_t* meta,
                                    const uint8_t* player_white, const uint16_t* actions, int8_t* out_boards,
                                    uint8_t* out_meta, int32_t* rewards, int32_t* status) {
    if (!e || !player_white || !actions || !out_boards || !out_meta || !rewards || !status) return fail("null argument");
    std::lock_guard<std::mutex> lk(e->mu);
    for (int i = 0; i < n; i++)
        if (actions[i] > A_QSB) return fail("action out of range at index " + std::to_string(i));
    if (eng_srv_use(e, n)) {
        if (!boards || !meta) return fail("null boards/meta");
        if (check_boards(1, boards)) return -1;
        if (eng_srv_call(e, ENG_NEXT, boards, meta, player_white[0] != 0, actions[0])) return -1;
        memcpy(out_boards, e->srv->out_board, 64);
        memcpy(out_meta, e->srv->out_meta, 8);
        rewards[0] = e->srv->reward;
        status[0] = e->srv->status;
        return 0;
    }
    if (devsrv_quiesce(e->device) || engine_reserve(e, n, 1)) return -1;
    // FIDE: the player argument is the side to move; reference: it only steers next_state's
    // promotion colour and rights logic (lib.rs:679-784), the state keeps current_player
    // the import reads side only under FIDE (the player argument is the side to move there)
    EngineLayout o;
    if (e->rules) {
        if (engine_upload(e, n, boards, meta, player_white, o, 1, actions)) return -1;
        SoA in{e->bb, e->meta, n}, out{e->bb2, e->meta2, n};
        k_fnext_state<<<grid_for(n), BLOCK, 0, e->stream>>>(in, e->acts, out, e->i32a, e->i32b);
        HIPCHK(hipGetLastError());
        engine_export(e, out);
    } else {  // one launch: import + next_state + export, in place on the staged mailbox
        if (n <= 0) return fail("n must be > 0");
        if (!boards || !meta) return fail("null boards/meta");
        if (check_boards(n, boards)) return -1;
        HIPCHK(hipSetDevice(e->device));
        if (engine_stage(e, n, 1, boards, meta, player_white, actions, o)) return -1;
        k_next_state_mb<<<grid_for(n), BLOCK, 0, e->stream>>>(e->mbox, e->m8, e->side, e->acts, n, e->i32a, e->i32b);
    }
    HIPCHK(hipGetLastError());
    if (engine_fetch(e, 0, o.i32b + (size_t)4 * n)) return -1;
    std::memcpy(out_boards, e->hio + o.mbox, (size_t)64 * n);
    std::memcpy(out_meta, e->hio + o.m8, (size_t)8 * n);
    std::memcpy(rewards, e->hio + o.i32a, (size_t)4 * n);
    std::memcpy(status, e->hio + o.i32b, (size_t)4 * n);
    return 0;
}

extern "C" int gc_engine_update_state(gc_engine* e, int n, const int8_t* boards, const uint8_t* meta,
                                      int8_t* out_boards, uint8_t* out_meta) {
    if (!e || !out_boards || !out_meta) return fail("null argument");
    std::lock_guard<std::mutex> lk(e->mu);
    if (eng_srv_use(e, n)) {
        if (!boards || !meta) return fail("null boards/meta");
        if (check_boards(1, boards)) return -1;
        if (eng_srv_call(e, ENG_UPDATE, boards, meta, false, 0)) return -1;
        memcpy(out_boards, e->srv->out_board, 64);
        memcpy(out_meta, e->srv->out_meta, 8);
        return 0;
    }
    if (devsrv_quiesce(e->device) || engine_reserve(e, n, 1)) return -1;
    EngineLayout o;
    if (engine_upload(e, n, boards, meta, nullptr, o)) return -1;
    SoA st{e->bb, e->meta, n};
    if (e->rules) k_fupdate_state<<<grid_for(n), BLOCK, 0, e->stream>>>(st);
    else k_update_state<<<grid_for(n), BLOCK, 0, e->stream>>>(st);
    HIPCHK(hipGetLastError());
    engine_export(e, st);
    HIPCHK(hipGetLastError());
    if (engine_fetch(e, 0, o.m8 + (size_t)8 * n)) return -1;
    std::memcpy(out_boards, e->hio + o.mbox, (size_t)64 * n);
    std::memcpy(out_meta, e->hio + o.m8, (size_t)8 * n);
    return 0;
}

// depth-3 subtrees as depth-2 ones: the level below `leaf` is materialised chunk by chunk
// (it is ~30x larger) and its nodes run in order of their move counts, so the leaf kernel's
// one remaining loop has (nearly) equal trip counts across a wave -- with depth-3 subtrees
// the inner loop's trip count varied per lane (PMC: ~60 % lane utilisation).
// leaf-kernel time of the split pass (gc_perft_leaf_stats): HIP events around every
// leaf launch (k_perft2_val / k_perft2_rec), on the stream it runs on; summed once the pass has synchronised
static std::mutex g_leaf_mu;
static uint64_t g_leaf_launches = 0, g_leaf_subtrees = 0, g_leaf_records = 0;
static double g_leaf_ms = 0.0;

static int perft_split_leaves(hipStream_t st, SoA leaf, uint64_t* leaf_out) {
    // parents per chunk 2^21 and up to 2^27 children (7.5 GiB of boards); GC_PERFT_CHUNK=k
    // (A/B): 2^k parents, 2^(k+6) children (2^20 / 2^22 measured 1.92 / 1.83 vs 1.93e12)
    static const int chunk_log2 = getenv("GC_PERFT_CHUNK") ? atoi(getenv("GC_PERFT_CHUNK")) : 21;
    // (the lead word holds a sorted position in RUN_LEN_SHIFT bits)
    if (chunk_log2 < 10 || chunk_log2 + 6 > RUN_LEN_SHIFT)
        return fail("GC_PERFT_CHUNK must be in [10, 21] (2^k parents per chunk)");
    const int64_t cap = (int64_t)1 << (chunk_log2 + 6);
    int chunk = 1 << chunk_log2;
    std::vector<hipEvent_t> evs;  // pairs around the leaf launches
    uint64_t subtrees = 0, records = 0;  // subtrees counted by the leaf kernel, of records made
    // GC_PERFT_DEDUP=0 (per call; tests): every record counted, transpositions too
    const char* dd = getenv("GC_PERFT_DEDUP");
    const bool dedup = !(dd && dd[0] == '0');
    int32_t *kc = nullptr, *offs = nullptr;
    uint8_t* bins = nullptr;
    u32 *hist = nullptr, *hbase = nullptr;
    const int max_blk = (chunk + BLOCK - 1) / BLOCK;
    const int max_dblk = (int)((cap + DEDUP_BLOCK * DEDUP_R - 1) / (DEDUP_BLOCK * DEDUP_R));  // the histograms' blocks
    const int hist_n = SPLIT_BINS * (dedup && max_dblk > max_blk ? max_dblk : max_blk);
    Node64* cr = nullptr;
    // the transposition pass: the records in expansion order; the sort's keys / values (16 B per
    // record), reused after it for the members' (leader, parent) pairs; the lead words; the
    // placed leaders' sorted positions
    Node64* cre = nullptr;
    u32* kv = nullptr;
    u32* leadw = nullptr;
    u32* spos = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    int rc = 0;
    std::string err;
    auto done = [&]() {
        void* ps[] = {kc, offs, cr, tmp, bins, hist, hbase, cre, kv, leadw, spos};
        for (void* q : ps) (void)hipFree(q);
        for (hipEvent_t ev : evs) (void)hipEventDestroy(ev);
    };
    if (dalloc(&kc, leaf.n) || dalloc(&offs, chunk) || dalloc(&cr, cap) || dalloc(&bins, cap) ||
        dalloc(&hist, (size_t)hist_n) || dalloc(&hbase, (size_t)hist_n) ||
        (dedup && (dalloc(&cre, cap) || dalloc(&kv, 4 * cap) || dalloc(&leadw, cap) || dalloc(&spos, cap)))) {
        done();
        return -1;
    }
    {  // scratch for the largest scan and sort of a chunk
        size_t b1 = 0, b2 = 0, b3 = 0;
        hipError_t he = hipcub::DeviceScan::ExclusiveSum(nullptr, b1, kc, offs, chunk, st);
        if (he == hipSuccess) he = hipcub::DeviceScan::ExclusiveSum(nullptr, b2, hist, hbase, hist_n, st);
        if (he == hipSuccess && dedup)
            he = hipcub::DeviceRadixSort::SortPairs(nullptr, b3, kv, kv + cap, kv + 2 * cap, kv + 3 * cap, (int)cap, 0, 32, st);
        tmp_bytes = b1 > b2 ? b1 : b2;
        tmp_bytes = tmp_bytes > b3 ? tmp_bytes : b3;
        if (he != hipSuccess) { done(); return fail(std::string("perft split: ") + hipGetErrorString(he)); }
        if (dalloc((char**)&tmp, tmp_bytes)) { done(); return -1; }
    }
    k_count_children<int32_t><<<grid_for(leaf.n), BLOCK, 0, st>>>(leaf, kc);
    for (int a = 0; a < leaf.n && rc == 0;) {
        int c = leaf.n - a < chunk ? leaf.n - a : chunk;
        size_t tb = tmp_bytes;
        hipError_t he = hipcub::DeviceScan::ExclusiveSum(tmp, tb, kc + a, offs, c, st);
        int32_t lo = 0, lc = 0;
        if (he == hipSuccess) he = hipMemcpyAsync(&lo, offs + c - 1, 4, hipMemcpyDeviceToHost, st);
        if (he == hipSuccess) he = hipMemcpyAsync(&lc, kc + a + c - 1, 4, hipMemcpyDeviceToHost, st);
        if (he == hipSuccess) he = hipStreamSynchronize(st);
        if (he != hipSuccess) { err = std::string("perft split: ") + hipGetErrorString(he); rc = -1; break; }
        int64_t total = (int64_t)lo + lc;
        if (total > cap) { chunk /= 2; continue; }  // an unusually bushy chunk: halve and retry
        he = hipMemsetAsync(leaf_out + a, 0, (size_t)8 * c, st);  // the parents' sums
        if (he != hipSuccess) { err = std::string("perft split: ") + hipGetErrorString(he); rc = -1; break; }
        unsigned long long* psum = reinterpret_cast<unsigned long long*>(leaf_out + a);
        if (total > 0 && dedup) {  // transpositions merged, the leaders binned and placed in order
            const int n = (int)total;
            const int nbd = (n + DEDUP_BLOCK * DEDUP_R - 1) / (DEDUP_BLOCK * DEDUP_R);
            k_expand_range_rec<<<grid_for(c), BLOCK, 0, st>>>(leaf, a, c, offs, cre);
            u32* const keys = kv;
            u32* const vals = kv + cap;
            u32* const keys2 = kv + 2 * cap;
            u32* const vals2 = kv + 3 * cap;
            uint2* const fw = reinterpret_cast<uint2*>(kv);  // after the sort: over keys | vals
            k_dedup_keys<<<grid_for(n), BLOCK, 0, st>>>(cre, n, keys, vals, bins);
            tb = tmp_bytes;
            he = hipcub::DeviceRadixSort::SortPairs(tmp, tb, keys, keys2, vals, vals2, n, 0, 32, st);
            if (he == hipSuccess) he = hipMemsetAsync(leadw, 0, (size_t)4 * n, st);
            if (he == hipSuccess) k_dedup_runs_f<<<grid_for(n), BLOCK, 0, st>>>(cre, n, keys2, vals2, leadw, fw);
            if (he == hipSuccess) k_leader_hist_f<<<nbd, DEDUP_BLOCK, 0, st>>>(n, leadw, bins, hist, nbd);
            tb = tmp_bytes;
            if (he == hipSuccess) he = hipcub::DeviceScan::ExclusiveSum(tmp, tb, hist, hbase, SPLIT_BINS * nbd, st);
            u32 hb = 0, hl = 0;  // the leaders: the last bin's base + its last block's count
            const size_t last = (size_t)SPLIT_BINS * nbd - 1;
            if (he == hipSuccess) he = hipMemcpyAsync(&hb, hbase + last, 4, hipMemcpyDeviceToHost, st);
            if (he == hipSuccess) he = hipMemcpyAsync(&hl, hist + last, 4, hipMemcpyDeviceToHost, st);
            if (he == hipSuccess) k_place_leaders_f<<<nbd, DEDUP_BLOCK, 0, st>>>(cre, n, bins, leadw, hbase, nbd, cr, spos);
            if (he == hipSuccess) he = hipStreamSynchronize(st);  // the leaf grid sized to the leaders
            if (he != hipSuccess) { err = std::string("perft split dedup: ") + hipGetErrorString(he); rc = -1; break; }
            const int lead_n = (int)(hb + hl);
            hipEvent_t e0 = nullptr, e1 = nullptr;
            if (hipEventCreate(&e0) == hipSuccess) evs.push_back(e0);
            if (hipEventCreate(&e1) == hipSuccess) evs.push_back(e1);
            if (e0 && e1) (void)hipEventRecord(e0, st);
            k_perft2_val<<<grid_for(lead_n), BLOCK, 0, st>>>(cr, lead_n, psum, n, keys2, fw, spos);
            if (e0 && e1) (void)hipEventRecord(e1, st);
            records += (uint64_t)total;
            subtrees += (uint64_t)lead_n;
        } else if (total > 0) {  // every record, in move-count order, then read in order
            const int nb = grid_for(c);
            k_expand_count<<<nb, BLOCK, 0, st>>>(leaf, a, c, bins, offs, hist, nb);
            tb = tmp_bytes;
            he = hipcub::DeviceScan::ExclusiveSum(tmp, tb, hist, hbase, SPLIT_BINS * nb, st);
            if (he != hipSuccess) { err = std::string("perft split scan: ") + hipGetErrorString(he); rc = -1; break; }
            k_expand_place<<<nb, BLOCK, 0, st>>>(leaf, a, c, bins, offs, hbase, nb, cr);
            hipEvent_t e0 = nullptr, e1 = nullptr;
            if (hipEventCreate(&e0) == hipSuccess) evs.push_back(e0);
            if (hipEventCreate(&e1) == hipSuccess) evs.push_back(e1);
            if (e0 && e1) (void)hipEventRecord(e0, st);
            k_perft2_rec<<<grid_for((int)total), BLOCK, 0, st>>>(cr, (int)total, psum);
            if (e0 && e1) (void)hipEventRecord(e1, st);
            records += (uint64_t)total;
            subtrees += (uint64_t)total;
        }
        he = hipGetLastError();
        if (he != hipSuccess) { err = std::string("perft split kernels: ") + hipGetErrorString(he); rc = -1; break; }
        a += c;
    }
    hipError_t he = hipStreamSynchronize(st);  // before the buffers are freed
    if (rc == 0 && he != hipSuccess) { err = std::string("perft split: ") + hipGetErrorString(he); rc = -1; }
    if (rc == 0) {
        double ms = 0.0;
        for (size_t k = 0; k + 1 < evs.size(); k += 2) {
            float t = 0.f;
            if (hipEventElapsedTime(&t, evs[k], evs[k + 1]) == hipSuccess) ms += t;
        }
        std::lock_guard<std::mutex> lk(g_leaf_mu);
        g_leaf_launches += evs.size() / 2;
        g_leaf_subtrees += subtrees;
        g_leaf_records += records;
        g_leaf_ms += ms;
    }
    done();
    return rc ? fail(err) : 0;
}

// which leaf pass ran, per pass (gc_perft_path_counts): tests assert that a configuration
// takes the path it is meant to pin
static std::atomic<unsigned long long> g_perft_path[4];  // split, sorted, small, fide

// Leaf level: perft(node, rem) of every node of `leaf` (rem <= 3, or few nodes) into out.
static int perft_leaf(hipStream_t st, SoA ls, int rem, uint64_t* out, int fide) {
    if (ls.n == 0) return 0;
    const char* sp = getenv("GC_PERFT_SPLIT");  // per call: tests compare both paths
    if (!fide && rem == 3 && ls.n >= 65536 && !(sp && sp[0] == '0')) {
        g_perft_path[0]++;
        return perft_split_leaves(st, ls, out);
    }
    if (!fide && rem >= 2 && ls.n >= 65536) {  // subtrees by root move count
        int32_t *kc = nullptr, *ks = nullptr, *ix = nullptr, *is = nullptr;
        void* tmp = nullptr;
        size_t tb = 0;
        hipError_t he = hipSuccess;
        if (dalloc(&kc, ls.n) || dalloc(&ks, ls.n) || dalloc(&ix, ls.n) || dalloc(&is, ls.n)) he = hipErrorOutOfMemory;
        if (he == hipSuccess) {
            k_count_children<int32_t><<<grid_for(ls.n), BLOCK, 0, st>>>(ls, kc);
            k_iota<<<grid_for(ls.n), BLOCK, 0, st>>>(ix, ls.n);
            he = hipcub::DeviceRadixSort::SortPairs(nullptr, tb, kc, ks, ix, is, ls.n, 0, 10, st);
        }
        if (he == hipSuccess && dalloc((char**)&tmp, tb) == 0)
            he = hipcub::DeviceRadixSort::SortPairs(tmp, tb, kc, ks, ix, is, ls.n, 0, 10, st);
        bool ok = he == hipSuccess && tmp;
        if (ok) {
            k_perft_small_perm<<<grid_for(ls.n), BLOCK, 0, st>>>(ls, is, rem, out);
            he = hipStreamSynchronize(st);  // before the temporaries are freed
        }
        (void)hipFree(tmp); (void)hipFree(kc); (void)hipFree(ks); (void)hipFree(ix); (void)hipFree(is);
        if (he != hipSuccess) return fail(std::string("perft sort: ") + hipGetErrorString(he));
        if (ok) { g_perft_path[1]++; return 0; }
    }
    g_perft_path[fide ? 3 : 2]++;
    if (fide) k_fperft_small<<<grid_for(ls.n), BLOCK, 0, st>>>(ls, rem, out);
    else k_perft_small<<<grid_for(ls.n), BLOCK, 0, st>>>(ls, rem, out);
    return 0;
}

// Children materialised per chunk of parents: <= PERFT_LEVEL_CAP nodes (60 B each plus
// 24 B of counts / offsets / values, ~11 GiB at 2^27) so any depth fits HBM; the split-leaf
// pass below holds its own <= 2^27-child chunk.  GC_PERFT_LEVEL_CAP (per call) lowers it so
// tests drive the chunked path at small sizes.
static const int64_t PERFT_LEVEL_CAP = (int64_t)1 << 27;

// out[i] = perft(nodes[i], rem).  While more than 3 plies remain, or while there are too few
// subtrees to fill the chip, the nodes are expanded into their children on the device
// (count, exclusive scan in 64 bits, write) and the children recursed on, one chunk of
// parents at a time when the level would not fit; the parents' values are the sums of their
// children's.  Sizes are 64-bit throughout: a level's child total may pass 2^31.
static int perft_nodes(hipStream_t st, SoA nodes, int rem, uint64_t* out, int fide) {
    if (nodes.n == 0) return 0;
    if (!(rem > 3 || (rem >= 2 && nodes.n < 131072))) return perft_leaf(st, nodes, rem, out, fide);
    int64_t cap = PERFT_LEVEL_CAP;
    if (const char* e = getenv("GC_PERFT_LEVEL_CAP")) cap = atoll(e) > 0 ? atoll(e) : cap;
    const int n = nodes.n;
    int64_t *cnt = nullptr, *offs = nullptr;
    u64* cb = nullptr;
    u32* cm = nullptr;
    uint64_t* cval = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    int64_t held = 0;  // children the buffers below can hold
    std::string err;
    auto release = [&]() {
        (void)hipStreamSynchronize(st);  // nothing in flight may still use the buffers
        void* ps[] = {cnt, offs, cb, cm, cval, tmp};
        for (void* q : ps) (void)hipFree(q);
        cb = nullptr; cm = nullptr; cval = nullptr;
    };
    if (dalloc(&cnt, n) || dalloc(&offs, n)) { release(); return -1; }
    if (fide) k_fcount_children<<<grid_for(n), BLOCK, 0, st>>>(nodes, cnt);
    else k_count_children<int64_t><<<grid_for(n), BLOCK, 0, st>>>(nodes, cnt);
    hipError_t he = hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, cnt, offs, n, st);
    if (he != hipSuccess || dalloc((char**)&tmp, tmp_bytes ? tmp_bytes : 1)) {
        release();
        return he != hipSuccess ? fail(std::string("perft scan: ") + hipGetErrorString(he)) : -1;
    }
    int chunk = n;
    for (int a = 0; a < n;) {
        const int c = n - a < chunk ? n - a : chunk;
        size_t tb = tmp_bytes;
        int64_t lo = 0, lc = 0;
        he = hipcub::DeviceScan::ExclusiveSum(tmp, tb, cnt + a, offs, c, st);
        if (he == hipSuccess) he = hipMemcpyAsync(&lo, offs + c - 1, 8, hipMemcpyDeviceToHost, st);
        if (he == hipSuccess) he = hipMemcpyAsync(&lc, cnt + a + c - 1, 8, hipMemcpyDeviceToHost, st);
        if (he == hipSuccess) he = hipStreamSynchronize(st);
        if (he != hipSuccess) { err = std::string("perft scan: ") + hipGetErrorString(he); break; }
        const int64_t total = lo + lc;
        if (total > cap && c > 1) { chunk = (c + 1) / 2; continue; }  // halve the chunk and rescan
        if (total >= ((int64_t)1 << 31)) { err = "perft: one node has too many children"; break; }
        if (total > held) {  // (re)allocate the child buffers for this chunk
            (void)hipStreamSynchronize(st);
            (void)hipFree(cb); (void)hipFree(cm); (void)hipFree(cval);
            cb = nullptr; cm = nullptr; cval = nullptr;
            held = 0;
            if (dalloc(&cb, (size_t)NBB * total) || dalloc(&cm, total) || dalloc(&cval, total)) { err = g_err; break; }
            held = total;
        }
        if (total > 0) {
            SoA ch{cb, cm, (int)total};
            if (fide) k_fexpand_range<<<grid_for(c), BLOCK, 0, st>>>(nodes, a, c, offs, ch);
            else k_expand_range<int64_t><<<grid_for(c), BLOCK, 0, st>>>(nodes, a, c, offs, ch);
            he = hipGetLastError();
            if (he != hipSuccess) { err = std::string("perft expand: ") + hipGetErrorString(he); break; }
            if (perft_nodes(st, ch, rem - 1, cval, fide)) { err = g_err; break; }
        }
        k_sum_children<int64_t><<<grid_for(c), BLOCK, 0, st>>>(offs, cnt + a, cval, c, out + a);
        he = hipGetLastError();
        if (he != hipSuccess) { err = std::string("perft sum: ") + hipGetErrorString(he); break; }
        a += c;
    }
    release();
    return err.empty() ? 0 : fail(err);
}

// perft over n roots (side to move = meta[0])
static int perft_device(hipStream_t st, SoA roots, int depth, uint64_t* d_out, int fide) {
    if (perft_nodes(st, roots, depth, d_out, fide)) return -1;
    hipError_t he = hipGetLastError();
    if (he == hipSuccess) he = hipStreamSynchronize(st);
    if (he != hipSuccess) return fail(std::string("perft kernels: ") + hipGetErrorString(he));
    return 0;
}

extern "C" int gc_perft_path_counts(uint64_t* out4) {
    if (!out4) return fail("null argument");
    for (int k = 0; k < 4; k++) out4[k] = g_perft_path[k].load();
    return 0;
}

extern "C" int gc_perft_leaf_stats(uint64_t* launches, uint64_t* subtrees, double* kernel_ms) {
    if (!launches || !subtrees || !kernel_ms) return fail("null argument");
    std::lock_guard<std::mutex> lk(g_leaf_mu);
    *launches = g_leaf_launches;
    *subtrees = g_leaf_subtrees;
    *kernel_ms = g_leaf_ms;
    return 0;
}

extern "C" int gc_perft_dedup_stats(uint64_t* records, uint64_t* counted) {
    if (!records || !counted) return fail("null argument");
    std::lock_guard<std::mutex> lk(g_leaf_mu);
    *records = g_leaf_records;
    *counted = g_leaf_subtrees;
    return 0;
}

extern "C" int gc_engine_perft(gc_engine* e, int n, const int8_t* boards, const uint8_t* meta, int depth,
                               uint64_t* nodes) {
    if (!e || !nodes) return fail("null argument");
    std::lock_guard<std::mutex> lk(e->mu);
    if (depth < 0 || depth > PERFT_MAXD) return fail("depth must be in [0, 8]");
    if (devsrv_quiesce(e->device) || engine_reserve(e, n, 1)) return -1;
    EngineLayout o;
    if (engine_upload(e, n, boards, meta, nullptr, o)) return -1;
    if (perft_device(e->stream, SoA{e->bb, e->meta, n}, depth, e->u64o, e->rules)) return -1;
    HIPCHK(hipMemcpyAsync(nodes, e->u64o, (size_t)8 * n, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return 0;
}

// ----------------------------------------------------------------------------- env API
#define GC_MAX_SUBSTREAMS 8
#ifndef GC_DEFAULT_STREAMS
#define GC_DEFAULT_STREAMS 2  // measured: 1 stream 10.2 us per ply, 2 streams 9.8, 3 10.6, 4 17 (graph-captured 11.4)
#endif
struct gc_env {
    int device = 0, n = 0;
    uint64_t seed = 0;
    hipStream_t stream = nullptr;
    EnvDev d{};
    u64* bb = nullptr; u32* meta = nullptr;
    int8_t* mbox = nullptr; uint8_t* m8 = nullptr; uint8_t* mask = nullptr;
    uint16_t* list = nullptr; int list_cap = 0; int32_t* counts = nullptr; u64* lmask = nullptr;
    uint64_t* stats = nullptr;
    hipEvent_t ev[8] = {};
    bool policy_ready = false;  // act[] holds policy picks for the current states
    int rules = 0;              // 0 reference, 1 FIDE (gc_fide.h)
    int8_t* ep = nullptr;       // FIDE ingest: en-passant files
    ApiOut* api_out = nullptr;  // the paired API step's output pointers (device copy of api_host)
    ApiOut api_host{};
    uint16_t* reset_acts = nullptr;
    EnvDev::InitCache* icd = nullptr;  // device copy of d.ic (the paired kernels read it from HBM)
    EnvDev::InitCache* icd_f = nullptr;  // the same for the FIDE reset position (gc_env_set_rules)
    uint16_t* racts_f = nullptr;
    OpenCache* open_cache = nullptr;     // a BLACK agent's openings (k_init_open_cache, gc_env_set_opponent)
    uint16_t* open_acts = nullptr;
    EnvDev::InitCache ic_f = {};
    uint8_t* slab = nullptr;  // per-board fields (Slab): bb, meta, hgen, draw, nsteps, reward, act, done, reason
    // Board-range streams of gc_env_step_random (gc_env_set_streams): ply p+1 of one range
    // depends only on ply p of the same range, so the ranges' launches interleave and the
    // launch ramp / tail of one range's ply overlaps another range's waves.
    int n_sub = 1;
    hipStream_t sub[GC_MAX_SUBSTREAMS] = {};
    hipEvent_t sub_ev[GC_MAX_SUBSTREAMS] = {};
    hipEvent_t fork_ev = nullptr;
    // the spill table of a BLACK agent's windows (gc_env.h; SpillTab): its slot counters are
    // copied to pinned host memory after every stepping call and checked before the next one
    int sp_bits = 0;
    u32* sp_ctr_h = nullptr;  // pinned: {slots claimed, failed}
    hipEvent_t sp_ev = nullptr;
    int sp_pending = 0;       // stepping calls since the last counter copy was read
    bool sp_failed = false;   // an insert failed: every stepping call fails until the windows are cleared
    gc_single_record* srec = nullptr;  // gc_env_single_call's host-mapped record
    gc_single_record* srec_d = nullptr;  // its device address
    // the quad rollout's completion word (EnvDev::InitCache::DoneWord): its host-mapped copy,
    // the launches issued so far, and the count the last gc_env_rollout_device call waits for
    // (0: the last call's work was not a quad launch -- gc_env_wait_rollout syncs the stream)
    u32* done_host = nullptr;
    u32* done_dev = nullptr;  // {ctr, seq}
    u32 done_issued = 0;
    u32 done_expect = 0;
    // the single-board server (k_single_server): its mailbox (host-mapped), stream, the launch
    // running (0: none), the last request served
    SrvBox* srv = nullptr;
    SrvBox* srv_d = nullptr;
    hipStream_t srv_stream = nullptr;
    u32 srv_launch = 0, srv_next_launch = 0, srv_seq = 0;
    int srv_board = -1;
};

static int srv_stop(gc_env* e);  // (the single-board server, below)
// before any launch on the env's device: no resident server (its own or another owner's) holds a queue
#define SRV_QUIESCE(e) do { if (devsrv_quiesce((e)->device)) return -1; } while (0)

static void env_free(gc_env* e) {
    void* ps[] = {e->api_out, e->reset_acts, e->icd, e->icd_f, e->racts_f, e->open_cache, e->open_acts, e->ep, e->slab, e->d.htab, e->mbox, e->m8, e->mask,
                  e->list, e->counts, e->lmask, e->stats};
    for (void* p : ps) if (p) (void)hipFree(p);
    for (auto& v : e->ev) if (v) (void)hipEventDestroy(v);
    for (int j = 0; j < GC_MAX_SUBSTREAMS; j++) {
        if (e->sub_ev[j]) (void)hipEventDestroy(e->sub_ev[j]);
        if (e->sub[j]) (void)hipStreamDestroy(e->sub[j]);
    }
    if (e->fork_ev) (void)hipEventDestroy(e->fork_ev);
    if (e->d.ic.spill.ent) (void)hipFree(e->d.ic.spill.ent);
    if (e->d.ic.spill.ctr) (void)hipFree(e->d.ic.spill.ctr);
    if (e->sp_ctr_h) (void)hipHostFree(e->sp_ctr_h);
    if (e->sp_ev) (void)hipEventDestroy(e->sp_ev);
    if (e->srec) (void)hipHostFree(e->srec);
    if (e->done_host) (void)hipHostFree(e->done_host);
    if (e->srv) (void)hipHostFree(e->srv);
    if (e->srv_stream) (void)hipStreamDestroy(e->srv_stream);
    if (e->done_dev) (void)hipFree(e->done_dev);
    if (e->stream) (void)hipStreamDestroy(e->stream);
}

// ----------------------------------------------------------------------------- spill table
// A BLACK agent's games have no move cap (chess_v2.py:291-292), so its 3-fold window is
// unbounded (saved_boards, chess_v2.py:192, 404-407).  Boards of a window past its per-board
// table's hist_cap go to the env's spill table (gc_env.h spill_find / spill_insert).  The
// host keeps the table's load under 1/4: after each stepping call the slot counters are
// copied to pinned memory; before the next call (or, when the copy has not landed, after at
// most SPILL_CHECK_LAG calls, synchronously) they are read, and a table past 1/4 is rehashed
// -- dead entries dropped, doubled when the live ones pass 1/8.  A failed insert (no free
// slot within SPILL_PROBES) sets a sticky flag: the next call reports it as an error, and so
// does every stepping call after it until every window is cleared (gc_env_reset of all
// boards, gc_env_set_states, gc_env_load), which starts a fresh table.
// Multi-step calls (gc_env_step_random, the fused rollouts) cannot wait for the next call:
// a launch's window generations are published only when it ends, so no entry it makes dead
// is reclaimed within it.  They run in chunks (spill_chunk): before each, the counters and a
// census of the windows within SPILL_PER_STEP x SPILL_CHUNK boards of the per-board cap are
// read, and the chunk is sized so that even if every such window spilled at every step the
// slots in use stay under half the table (rehashed / doubled first when that leaves fewer
// than SPILL_CHUNK_MIN steps).
#define SPILL_CHECK_LAG 4
#define SPILL_CHUNK 128      // steps per launch of a spill-enabled multi-step call, at most
#define SPILL_CHUNK_MIN 16   // below this many steps of room the table is rehashed / doubled first
#define SPILL_PER_STEP 2     // window boards one step adds: the agent's and the opponent's pre-move boards
#define SPILL_BITS_MAX 30    // 2^30 entries = 64 GiB

// boards whose window is within SPILL_PER_STEP x SPILL_CHUNK boards of the per-board cap
__global__ void k_spill_census(const u32* __restrict__ meta, int n, u32 thresh, u32* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool near = i < n && hl_of(meta[i]) >= thresh;
    const unsigned long long b = __ballot(near);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(out, (u32)__popcll(b));
}

__global__ void k_spill_rehash(const u64* __restrict__ old, u32 old_mask, SpillTab nt, const u32* __restrict__ hgen) {
    const size_t slot = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (slot > old_mask) return;
    const u64* e = old + slot * 8;
    const u64 hdr = e[0];
    const u32 o1 = sp_owner1(hdr);
    if (o1 == 0 || sp_gen(hdr) != hgen[o1 - 1]) return;  // empty or dead
    Pos b = {e[1], e[2], e[3], e[4], e[5], e[6], e[7], 0};
    DevHist h{nullptr, const_cast<u32*>(hgen), sp_gen(hdr), (int)(o1 - 1), HTAB_BITS_UNCAPPED};
    h.sp = nt;
    u32 t = sp_home(board_key(b), o1 - 1, nt.mask);
    for (int probe = 0; probe < SPILL_PROBES; probe++, t = (t + 1) & nt.mask) {
        u64 z = 0;
        if (h.sp_cas(t, z, hdr)) {
            h.sp_put(t, b);
            h.sp_claimed();
            return;
        }
    }
    h.sp_fail();
}

static int spill_bits_max() {
    const char* v = getenv("GC_SPILL_BITS_MAX");  // tests: cap the growth to force a failed insert
    return v && atoi(v) >= 6 && atoi(v) < SPILL_BITS_MAX ? atoi(v) : SPILL_BITS_MAX;
}

static int spill_bits_for(int n) {
    int b = 14;
    while (b < 22 && (1 << (b - 4)) < n) b++;  // 2^20 entries (64 MiB) at 65 536 boards
    const char* v = getenv("GC_SPILL_BITS");   // tests: start small to drive the rehash / growth path
    if (v && atoi(v) >= 6 && atoi(v) <= 30) b = atoi(v);
    return b;
}

// publish e->d.ic.spill to the device copy the paired kernels read
static int spill_publish(gc_env* e) {
    HIPCHK(hipMemcpyAsync(&e->icd->spill, &e->d.ic.spill, sizeof(SpillTab), hipMemcpyHostToDevice, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return 0;
}

static int spill_alloc(gc_env* e, int bits) {
    SpillTab t = {nullptr, nullptr, (1u << bits) - 1};
    if (dalloc(&t.ent, (size_t)8 << bits)) return -1;
    if (dalloc(&t.ctr, 4)) { (void)hipFree(t.ent); return -1; }
    hipError_t he = hipMemsetAsync(t.ent, 0, (size_t)64 << bits, e->stream);
    if (he == hipSuccess) he = hipMemsetAsync(t.ctr, 0, 16, e->stream);
    if (he == hipSuccess && !e->sp_ctr_h) he = hipHostMalloc(&e->sp_ctr_h, 16, hipHostMallocDefault);
    if (he == hipSuccess && !e->sp_ev) he = hipEventCreateWithFlags(&e->sp_ev, hipEventDisableTiming);
    if (he != hipSuccess) { (void)hipFree(t.ent); (void)hipFree(t.ctr); return fail(std::string("spill table: ") + hipGetErrorString(he)); }
    if (e->d.ic.spill.ent) (void)hipFree(e->d.ic.spill.ent);
    if (e->d.ic.spill.ctr) (void)hipFree(e->d.ic.spill.ctr);
    e->d.ic.spill = t;
    e->sp_bits = bits;
    e->sp_pending = 0;
    e->sp_failed = false;
    e->sp_ctr_h[0] = e->sp_ctr_h[1] = e->sp_ctr_h[2] = 0;
    return spill_publish(e);
}

static void spill_drop(gc_env* e) {
    if (e->d.ic.spill.ent) (void)hipFree(e->d.ic.spill.ent);
    if (e->d.ic.spill.ctr) (void)hipFree(e->d.ic.spill.ctr);
    e->d.ic.spill = SpillTab{nullptr, nullptr, 0};
    e->sp_bits = 0;
    e->sp_pending = 0;
}

// rehash the live entries into a table of 2^bits slots (the stream is idle)
static int spill_rehash(gc_env* e, int bits) {
    const SpillTab old = e->d.ic.spill;
    SpillTab t = {nullptr, nullptr, (1u << bits) - 1};
    if (dalloc(&t.ent, (size_t)8 << bits)) return -1;
    if (dalloc(&t.ctr, 4)) { (void)hipFree(t.ent); return -1; }
    u32 c[2] = {0, 0};
    hipError_t he = hipMemsetAsync(t.ent, 0, (size_t)64 << bits, e->stream);
    if (he == hipSuccess) he = hipMemsetAsync(t.ctr, 0, 16, e->stream);
    if (he == hipSuccess) {
        const size_t slots = (size_t)old.mask + 1;
        k_spill_rehash<<<(unsigned)((slots + BLOCK - 1) / BLOCK), BLOCK, 0, e->stream>>>(old.ent, old.mask, t, e->d.hgen);
        he = hipGetLastError();
    }
    if (he == hipSuccess) he = hipMemcpyAsync(c, t.ctr, 8, hipMemcpyDeviceToHost, e->stream);
    if (he == hipSuccess) he = hipStreamSynchronize(e->stream);
    if (he != hipSuccess || c[1]) {
        (void)hipFree(t.ent); (void)hipFree(t.ctr);
        return fail(he != hipSuccess ? std::string("spill rehash: ") + hipGetErrorString(he)
                                     : std::string("spill rehash: no free slot (table of 2^") + std::to_string(bits) + ")");
    }
    (void)hipFree(old.ent);
    (void)hipFree(old.ctr);
    e->d.ic.spill = t;
    e->sp_bits = bits;
    e->sp_pending = 0;
    e->sp_ctr_h[0] = c[0];
    e->sp_ctr_h[1] = 0;
    return spill_publish(e);
}

static int spill_failed(gc_env* e) {
    e->sp_failed = true;
    return fail("repetition spill table: an insert found no free slot (a window outgrew 2^" + std::to_string(e->sp_bits) +
                " shared entries); results since then are invalid until every window is cleared (gc_env_reset of all "
                "boards, gc_env_set_states or gc_env_load)");
}

// every window was cleared (the stream is idle): a failed table starts afresh
static int spill_windows_cleared(gc_env* e) {
    if (!e->d.ic.spill.ent || !e->sp_failed) return 0;
    return spill_alloc(e, e->sp_bits);
}

// before a stepping call: the counters of the last copy that landed
static int spill_before(gc_env* e) {
    if (!e->d.ic.spill.ent) return 0;
    if (e->sp_failed) return spill_failed(e);
    if (!e->sp_pending) return 0;
    if (e->sp_pending >= SPILL_CHECK_LAG) HIPCHK(hipEventSynchronize(e->sp_ev));
    else if (hipEventQuery(e->sp_ev) != hipSuccess) return 0;  // not landed yet: check next call
    e->sp_pending = 0;
    const u32 used = e->sp_ctr_h[0], failed = e->sp_ctr_h[1];
    if (failed) return spill_failed(e);
    const u32 cap = 1u << e->sp_bits;
    if (used > cap / 4) {
        HIPCHK(hipStreamSynchronize(e->stream));
        if (spill_rehash(e, e->sp_bits)) return -1;  // drops the dead entries
        if (e->sp_ctr_h[0] > cap / 8 && e->sp_bits < spill_bits_max() && spill_rehash(e, e->sp_bits + 1)) return -1;
    }
    return 0;
}

// the steps the next launch of a multi-step call may take (<= want; synchronous): see above
static int spill_chunk(gc_env* e, int want) {
    if (!e->d.ic.spill.ent || want <= 0) return want;
    if (e->sp_failed) return spill_failed(e);
    const u32 thresh = (u32)(hist_cap(HTAB_BITS_UNCAPPED) - SPILL_PER_STEP * SPILL_CHUNK);
    bool rehashed = false;
    for (;;) {
        u32* ctr = e->d.ic.spill.ctr;
        HIPCHK(hipMemsetAsync(ctr + 2, 0, 4, e->stream));
        k_spill_census<<<grid_for(e->n), BLOCK, 0, e->stream>>>(e->d.st.meta, e->n, thresh, ctr + 2);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(e->sp_ctr_h, ctr, 12, hipMemcpyDeviceToHost, e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));
        e->sp_pending = 0;
        const u32 used = e->sp_ctr_h[0], near = e->sp_ctr_h[2];
        if (e->sp_ctr_h[1]) return spill_failed(e);
        const uint64_t half = (uint64_t)1 << (e->sp_bits - 1);
        const uint64_t room = half > used ? half - used : 0;
        uint64_t steps = near ? room / ((uint64_t)SPILL_PER_STEP * near) : (uint64_t)SPILL_CHUNK;
        if (steps > SPILL_CHUNK) steps = SPILL_CHUNK;
        if (steps > (uint64_t)want) steps = (uint64_t)want;
        const uint64_t enough = want < SPILL_CHUNK_MIN ? (uint64_t)want : (uint64_t)SPILL_CHUNK_MIN;
        if (steps >= enough) return (int)steps;
        if (e->sp_bits >= spill_bits_max()) {
            if (steps >= 1 || rehashed) return steps >= 1 ? (int)steps : 1;  // (a failed insert would be reported)
            if (spill_rehash(e, e->sp_bits)) return -1;  // the dead entries, at least
            rehashed = true;
            continue;
        }
        // too little room: drop the dead entries first, then double
        if (spill_rehash(e, rehashed ? e->sp_bits + 1 : e->sp_bits)) return -1;
        rehashed = true;
    }
}

// after a stepping call: copy the counters (asynchronously) for the next check
static int spill_after(gc_env* e) {
    if (!e->d.ic.spill.ent) return 0;
    HIPCHK(hipMemcpyAsync(e->sp_ctr_h, e->d.ic.spill.ctr, 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipEventRecord(e->sp_ev, e->stream));
    e->sp_pending++;
    return 0;
}

// the spill table's state (synchronous): log2 slots (0: none), slots in use (live + dead),
// live entries
__global__ void k_spill_live(const u64* __restrict__ ent, u32 mask, const u32* __restrict__ hgen,
                             unsigned long long* __restrict__ live) {
    const size_t slot = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (slot > mask) return;
    const u64 hdr = ent[slot * 8];
    const u32 o1 = sp_owner1(hdr);
    if (o1 != 0 && sp_gen(hdr) == hgen[o1 - 1]) atomicAdd(live, 1ull);
}
extern "C" int gc_env_spill_info(gc_env* e, int* bits, uint64_t* used, uint64_t* live) {
    if (!e || !bits || !used || !live) return fail("null argument");
    SRV_QUIESCE(e);
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    *bits = e->sp_bits;
    *used = *live = 0;
    const SpillTab& sp = e->d.ic.spill;
    if (!sp.ent) return 0;
    unsigned long long* d = nullptr;
    if (dalloc(&d, 1)) return -1;
    u32 c[2] = {0, 0};
    unsigned long long lv = 0;
    hipError_t he = hipMemsetAsync(d, 0, 8, e->stream);
    if (he == hipSuccess) {
        const size_t slots = (size_t)sp.mask + 1;
        k_spill_live<<<(unsigned)((slots + BLOCK - 1) / BLOCK), BLOCK, 0, e->stream>>>(sp.ent, sp.mask, e->d.hgen, d);
        he = hipGetLastError();
    }
    if (he == hipSuccess) he = hipMemcpyAsync(&lv, d, 8, hipMemcpyDeviceToHost, e->stream);
    if (he == hipSuccess) he = hipMemcpyAsync(c, sp.ctr, 8, hipMemcpyDeviceToHost, e->stream);
    if (he == hipSuccess) he = hipStreamSynchronize(e->stream);
    (void)hipFree(d);
    if (he != hipSuccess) return fail(std::string("spill info: ") + hipGetErrorString(he));
    *used = c[0];
    *live = lv;
    if (c[1]) return fail("repetition spill table: an insert found no free slot");
    return 0;
}

// The repetition tables for move-capped games (HTAB_BITS) or for a BLACK agent's uncapped
// ones (HTAB_BITS_UNCAPPED + the spill table); the stream is idle, the windows are cleared.
static int set_window_kind(gc_env* e, bool uncapped) {
    const int bits = uncapped ? HTAB_BITS_UNCAPPED : HTAB_BITS;
    if (bits != e->d.hbits) {
        size_t nb64 = ((size_t)e->n + 63) / 64 * 64;
        u64* t = nullptr;
        if (dalloc(&t, ((size_t)8 << bits) * nb64)) return -1;
        HIPCHK(hipMemsetAsync(t, 0, ((size_t)64 << bits) * nb64, e->stream));
        (void)hipFree(e->d.htab);
        e->d.htab = t;
        e->d.hbits = bits;
    }
    if (uncapped && !e->d.ic.spill.ent) {  // a BLACK agent's windows may outgrow the table
        if (spill_alloc(e, spill_bits_for(e->n))) return -1;
    } else if (!uncapped && e->d.ic.spill.ent) {
        HIPCHK(hipStreamSynchronize(e->stream));
        spill_drop(e);
        if (spill_publish(e)) return -1;
    }
    return 0;
}

// kernel dispatch on the env's opponent mode (a kernel-argument-uniform choice made once per
// launch on the host, so the opponent="none" kernels carry no opponent code)
static void launch_reset(gc_env* e, const uint8_t* mask, int select) {
    if (e->rules && e->d.opp) k_fenv_reset<true><<<grid_for(e->n), BLOCK, 0, e->stream>>>(e->d, mask, select);
    else if (e->rules) k_fenv_reset<false><<<grid_for(e->n), BLOCK, 0, e->stream>>>(e->d, mask, select);
    else if (e->d.opp) k_env_reset<true><<<grid_for(e->n), BLOCK, 0, e->stream>>>(e->d, mask, select);
    else k_env_reset<false><<<grid_for(e->n), BLOCK, 0, e->stream>>>(e->d, mask, select);
}
template <bool POLICY>
static void launch_step(gc_env* e) {
    if (e->rules && e->d.opp) k_fenv_step<POLICY, true><<<grid_for(e->n), BLOCK, 0, e->stream>>>(e->d);
    else if (e->rules) k_fenv_step<POLICY, false><<<grid_for(e->n), BLOCK, 0, e->stream>>>(e->d);
    else if (e->d.opp) k_env_step<POLICY, true><<<grid_for(e->n), BLOCK, 0, e->stream>>>(e->d);
    else k_env_step<POLICY, false><<<grid_for(e->n), BLOCK, 0, e->stream>>>(e->d);
}

// the reset position's cache of the env's rules (reference or FIDE) for the paired kernels
struct ResetInfo {
    const EnvDev::InitCache* icd;
    const uint16_t* racts;
    u32 rinfo;  // table << 16 | total
};
static ResetInfo reset_info(const gc_env* e) {
    const EnvDev::InitCache& ic = e->rules ? e->ic_f : e->d.ic;
    return ResetInfo{e->rules ? e->icd_f : e->icd, e->rules ? e->racts_f : e->d.reset_acts,
                     (ic.table ? 1u << 16 : 0u) | (u32)(ic.total & 0xFFFF)};
}

// The paired kernels serve opponent "none" (both rules) and the random opponent when the
// start position's picks come from its table and, for a BLACK agent, no opening can end in
// both kings checked (pair_step_vs); otherwise the one-wave kernels run.
// the reset picks of the self-play policy (reference rules): the move-set order table
static const uint16_t* sw_table(const ResetInfo& r) {
    return r.racts ? r.racts + RESET_ACTS_MAX : r.racts;
}
static bool pair_ok(const gc_env* e) {
    if (!e->d.opp) return true;
    if (e->rules) return false;  // FIDE with the random opponent: the one-wave kernels (k_fenv_*)
    const EnvDev::InitCache& ic = e->d.ic;
    return ic.usable && ic.table && (!e->d.agent_black || ic.open_safe);
}
static int pair_opp(const gc_env* e) { return e->d.opp ? (e->d.agent_black ? 2 : 1) : 0; }

// one ply (opponent: one two-ply step) of the paired step kernel over the board blocks
// [b0, b0 + nb) (64 boards each)
static void launch_step2(gc_env* e, hipStream_t st, int b0 = 0, int nb = -1) {
    const EnvDev& d = e->d;
    const ResetInfo r = reset_info(e);
    const int per_wg = PAIR_BOARDS * PAIRS_WG;
    if (nb < 0) nb = (e->n + PAIR_BOARDS - 1) / PAIR_BOARDS;
    const dim3 grid((nb + PAIRS_WG - 1) / PAIRS_WG), block(2 * per_wg);
    switch (e->rules ? 3 : pair_opp(e)) {
        case 3: k_env_step2<true><<<grid, block, 0, st>>>(e->slab, d.n, b0, d.seed, d.htab, r.racts, r.icd, r.rinfo); break;
        case 0: k_env_step2<false><<<grid, block, 0, st>>>(e->slab, d.n, b0, d.seed, d.htab, sw_table(r), r.icd, r.rinfo); break;
        case 1: k_env_step2<false, 1><<<grid, block, 0, st>>>(e->slab, d.n, b0, d.seed, d.htab, sw_table(r), r.icd, r.rinfo); break;
        default: k_env_step2<false, 2><<<grid, block, 0, st>>>(e->slab, d.n, b0, d.seed, d.htab, sw_table(r), r.icd, r.rinfo); break;
    }
}

extern "C" int gc_env_create(int device, int n_boards, uint64_t seed, const int8_t* initial_board, gc_env** out) {
    if (!out) return fail("null out pointer");
    if (n_boards <= 0) return fail("n_boards must be > 0");
    int nd = 0;
    HIPCHK(hipGetDeviceCount(&nd));
    if (device < 0 || device >= nd) return fail("device index out of range");
    static const int8_t DEF[64] = {-3, -5, -4, -2, -1, -4, -5, -3, -6, -6, -6, -6, -6, -6, -6, -6,
                                   0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,
                                   0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,
                                   6,  6,  6,  6,  6,  6,  6,  6,  3,  5,  4,  2,  1,  4,  5,  3};
    const int8_t* ib = initial_board ? initial_board : DEF;
    if (check_boards(1, ib)) return -1;
    gc_env* e = new gc_env();
    e->device = device;
    e->n = n_boards;
    e->seed = seed;
    int n = n_boards;
    size_t nb64 = ((size_t)n + 63) / 64 * 64;  // the window tables come in blocks of 64 boards
    hipError_t he = hipSetDevice(device);
    if (he == hipSuccess) he = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking);
    if (he != hipSuccess) { env_free(e); delete e; return fail(std::string("stream: ") + hipGetErrorString(he)); }
    if (dalloc(&e->slab, Slab::BYTES_PER_BOARD * (size_t)n) ||
        dalloc(&e->d.htab, (size_t)HTAB * 8 * nb64) || dalloc(&e->mbox, (size_t)64 * n) ||
        dalloc(&e->m8, (size_t)8 * n) || dalloc(&e->mask, n) || dalloc(&e->counts, n) || dalloc(&e->stats, (size_t)8 * n + 8) /* [n][8] + the 8 sums */) {
        std::string m = g_err;
        env_free(e); delete e;
        return fail(m);
    }
    {
        uint8_t* sl = e->slab;
        size_t nz = (size_t)n;
        e->bb = reinterpret_cast<u64*>(sl);
        e->meta = reinterpret_cast<u32*>(sl + Slab::meta(nz));
        e->d.hgen = reinterpret_cast<u32*>(sl + Slab::hgen(nz));
        e->d.draw = reinterpret_cast<u32*>(sl + Slab::draw(nz));
        e->d.nsteps = reinterpret_cast<u32*>(sl + Slab::nsteps(nz));
        e->d.reward = reinterpret_cast<int32_t*>(sl + Slab::reward(nz));
        e->d.act = reinterpret_cast<uint16_t*>(sl + Slab::act(nz));
        e->d.done = sl + Slab::done(nz);
        e->d.reason = sl + Slab::reason(nz);
    }
    // initial board bitboards (pure data conversion of the caller's input; no engine work)
    Pos ip = from_mailbox(ib, 0);
    u64 ibb[NBB] = {ip.k, ip.q, ip.r, ip.b, ip.n, ip.p, ip.w};
    for (int j = 0; j < NBB; j++) e->d.init[j] = ibb[j];
    he = hipSuccess;
    if (he == hipSuccess) he = hipMemsetAsync(e->d.draw, 0, (size_t)4 * n, e->stream);
    if (he == hipSuccess) he = hipMemsetAsync(e->d.htab, 0, (size_t)64 * HTAB * nb64, e->stream);
    if (he == hipSuccess) he = hipMemsetAsync(e->d.hgen, 0, (size_t)4 * n, e->stream);
    if (he == hipSuccess) he = hipMemsetAsync(e->d.nsteps, 0, (size_t)4 * n, e->stream);
    if (he == hipSuccess) he = hipMemsetAsync(e->d.reward, 0, (size_t)4 * n, e->stream);
    if (he == hipSuccess) he = hipMemsetAsync(e->d.done, 0, (size_t)n, e->stream);
    if (he == hipSuccess) he = hipMemsetAsync(e->d.reason, 0, (size_t)n, e->stream);
    if (he == hipSuccess) he = hipMemsetAsync(e->stats, 0, (size_t)64 * n, e->stream);
    for (auto& v : e->ev) if (he == hipSuccess) he = hipEventCreate(&v);
    if (he != hipSuccess) { env_free(e); delete e; return fail(std::string("env init: ") + hipGetErrorString(he)); }
    e->d.st = SoA{e->bb, e->meta, n};
    e->d.seed = seed;
    e->d.n = n;
    e->d.opp = 0;
    e->d.agent_black = 0;
    e->d.hbits = HTAB_BITS;
    {  // the start position's move set, shared by every reset (EnvDev::ic)
        EnvDev::InitCache* dic = nullptr;
        uint16_t* dacts = nullptr;
        if (dalloc(&dic, 1) || dalloc(&dacts, 2 * RESET_ACTS_MAX)) {
            std::string m = g_err; (void)hipFree(dic); env_free(e); delete e; return fail(m);
        }
        e->reset_acts = dacts;
        e->d.reset_acts = dacts;
        e->icd = dic;
        k_init_cache<<<1, BLOCK, 0, e->stream>>>(e->d, dic, dacts);
        he = hipGetLastError();
        if (he == hipSuccess) he = hipMemcpyAsync(&e->d.ic, dic, sizeof(EnvDev::InitCache), hipMemcpyDeviceToHost, e->stream);
        if (he == hipSuccess) he = hipStreamSynchronize(e->stream);
        if (he != hipSuccess) { env_free(e); delete e; return fail(std::string("init cache: ") + hipGetErrorString(he)); }
        // the completion word of the quad rollout (host-mapped, fine-grained)
        u32* hw = nullptr;
        he = hipHostMalloc(&hw, 4, hipHostMallocMapped | hipHostMallocCoherent);
        if (he == hipSuccess) { e->done_host = hw; *hw = 0; he = hipMalloc(&e->done_dev, 8); }
        if (he == hipSuccess) he = hipMemsetAsync(e->done_dev, 0, 8, e->stream);
        u32* hwd = nullptr;
        if (he == hipSuccess) he = hipHostGetDevicePointer((void**)&hwd, hw, 0);
        if (he == hipSuccess) {
            e->d.ic.done = EnvDev::InitCache::DoneWord{e->done_dev, e->done_dev + 1, hwd};
            he = hipMemcpyAsync(&dic->done, &e->d.ic.done, sizeof(e->d.ic.done), hipMemcpyHostToDevice, e->stream);
        }
        if (he == hipSuccess) he = hipStreamSynchronize(e->stream);
        if (he != hipSuccess) { env_free(e); delete e; return fail(std::string("completion word: ") + hipGetErrorString(he)); }
    }
    launch_reset(e, nullptr, 1);
    he = hipGetLastError();
    if (he == hipSuccess) he = hipStreamSynchronize(e->stream);
    if (he != hipSuccess) { env_free(e); delete e; return fail(std::string("reset: ") + hipGetErrorString(he)); }
    e->policy_ready = true;
    {
        const char* sv = getenv("GC_STREAMS");
        int k = sv ? atoi(sv) : GC_DEFAULT_STREAMS;
        if (k > 1 && gc_env_set_streams(e, k)) { std::string m = g_err; env_free(e); delete e; return fail(m); }
    }
    *out = e;
    return 0;
}

// opponent mode (chess_v2.py:133-181): opponent 0 "none", 1 "random" (the device policy
// answers inside every step); agent_white 0 = player_color BLACK (requires an opponent: the
// reference's reset calls the opponent policy to open).  Resets every board.
extern "C" int gc_env_set_opponent(gc_env* e, int opponent, int agent_white) {
    if (!e) return fail("null env");
    SRV_QUIESCE(e);
    if (opponent != 0 && opponent != 1) return fail("opponent must be 0 (none) or 1 (random)");
    if (!agent_white && !opponent) return fail("player_color BLACK needs an opponent (chess_v2.py:208-212)");
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    if (set_window_kind(e, !agent_white)) return -1;
    e->d.opp = opponent;
    e->d.agent_black = agent_white ? 0 : 1;
    if (!agent_white && e->d.ic.table && !e->open_cache) {  // the openings of a BLACK agent's resets
        if (dalloc(&e->open_cache, RESET_ACTS_MAX) || dalloc(&e->open_acts, (size_t)RESET_ACTS_MAX * RESET_ACTS_MAX))
            return -1;
        k_init_open_cache<<<(RESET_ACTS_MAX + BLOCK - 1) / BLOCK, BLOCK, 0, e->stream>>>(
            e->d, e->icd, e->reset_acts + RESET_ACTS_MAX, e->open_cache, e->open_acts);
        HIPCHK(hipGetLastError());
        e->d.ic.open = e->open_cache;
        e->d.ic.open_acts = e->open_acts;
        HIPCHK(hipMemcpyAsync(&e->icd->open, &e->d.ic.open, sizeof(e->d.ic.open) + sizeof(e->d.ic.open_acts),
                              hipMemcpyHostToDevice, e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));
    }
    HIPCHK(hipMemsetAsync(e->d.draw, 0, (size_t)4 * e->n, e->stream));  // fresh policy streams
    launch_reset(e, nullptr, 1);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(e->stream));
    e->policy_ready = true;
    return 0;
}

// rules 0: the reference's (default); 1: FIDE (gc_fide.h; with the random opponent on the
// one-wave kernels).  Resets every board and restarts the policy streams.
extern "C" int gc_env_set_rules(gc_env* e, int rules) {
    if (!e) return fail("null env");
    SRV_QUIESCE(e);
    if (rules != 0 && rules != 1) return fail("rules must be 0 (reference) or 1 (fide)");
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    if (rules && !e->icd_f) {  // the FIDE reset position's move set (paired kernels)
        if (dalloc(&e->icd_f, 1) || dalloc(&e->racts_f, RESET_ACTS_MAX)) return -1;
        k_finit_cache<<<1, BLOCK, 0, e->stream>>>(e->d, e->icd_f, e->racts_f);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(&e->ic_f, e->icd_f, sizeof(EnvDev::InitCache), hipMemcpyDeviceToHost, e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));
    }
    e->rules = rules;
    HIPCHK(hipMemsetAsync(e->d.draw, 0, (size_t)4 * e->n, e->stream));
    launch_reset(e, nullptr, 1);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(e->stream));
    e->policy_ready = true;
    return 0;
}

extern "C" int gc_env_destroy(gc_env* e) {
    if (!e) return 0;
    (void)hipSetDevice(e->device);
    (void)srv_stop(e);
    srv_unregister(e);
    (void)hipStreamSynchronize(e->stream);
    env_free(e);
    delete e;
    return 0;
}

extern "C" int gc_env_num_boards(gc_env* e) { return e ? e->n : -1; }

extern "C" int gc_env_reset(gc_env* e, const uint8_t* mask) {
    if (!e) return fail("null env");
    SRV_QUIESCE(e);
    HIPCHK(hipSetDevice(e->device));
    if (mask) HIPCHK(hipMemcpyAsync(e->mask, mask, e->n, hipMemcpyHostToDevice, e->stream));
    launch_reset(e, mask ? e->mask : nullptr, 1);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(e->stream));
    if (!mask && spill_windows_cleared(e)) return -1;
    e->policy_ready = true;
    return 0;
}

// ---- single-board env ops (k_single)
extern "C" int gc_env_single_setup(gc_env* e, int agent_white) {
    if (!e) return fail("null env");
    SRV_QUIESCE(e);
    if (e->rules) return fail("the single-board env ops follow the reference's rules");
    if (e->d.opp) return fail("the single-board env ops drive the opponent from the host (opponent 0)");
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    if (set_window_kind(e, !agent_white)) return -1;
    if (!e->srec) {
        HIPCHK(hipHostMalloc(&e->srec, sizeof(gc_single_record), hipHostMallocMapped));
        HIPCHK(hipHostGetDevicePointer((void**)&e->srec_d, e->srec, 0));
    }
    return 0;
}

// ---- the single-board server's host side
static bool srv_enabled() {
    static const bool off = getenv("GC_SINGLE_SERVER") && atoi(getenv("GC_SINGLE_SERVER")) == 0;
    return !off;
}
// stop the server (if one runs) and wait until it has drained: every other op on this env
// reads or writes the board's memory through other kernels
static int srv_stop(gc_env* e) {
    DevSrv& s = devsrv(e->device);
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    devsrv_release(s, e);
    if (!e->srv_launch) return 0;
    SrvBox* b = e->srv;
    __atomic_store_n(&b->op, (u32)SRV_QUIT, __ATOMIC_RELAXED);
    __atomic_store_n(&b->req_seq, e->srv_seq + 1, __ATOMIC_RELEASE);  // (never served: QUIT)
    const hipError_t he = hipStreamSynchronize(e->srv_stream);
    __atomic_store_n(&b->req_seq, e->srv_seq, __ATOMIC_RELEASE);
    e->srv_launch = 0;
    if (he != hipSuccess) return fail(std::string("single-board server: ") + hipGetErrorString(he));
    return 0;
}
// one op through the server (started on demand); the record lands in e->srec
static int srv_stop_v(void* e) { return srv_stop(static_cast<gc_env*>(e)); }
static int srv_call(gc_env* e, int board, int op, int action, int flags) {
    HIPCHK(hipSetDevice(e->device));
    DevSrv& s = devsrv(e->device);
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    if (devsrv_claim(s, e, srv_stop_v)) return -1;
    if (!e->srv) {
        HIPCHK(hipHostMalloc(&e->srv, sizeof(SrvBox), hipHostMallocMapped | hipHostMallocCoherent));
        memset(e->srv, 0, sizeof(SrvBox));
        HIPCHK(hipHostGetDevicePointer((void**)&e->srv_d, e->srv, 0));
        HIPCHK(hipStreamCreateWithFlags(&e->srv_stream, hipStreamNonBlocking));
    }
    if (e->srv_launch && e->srv_board != board && (srv_stop(e) || devsrv_claim(s, e, srv_stop_v))) return -1;
    SrvBox* b = e->srv;
    const u32 seq = e->srv_seq + 1;
    __atomic_store_n(&b->op, (u32)op, __ATOMIC_RELAXED);
    __atomic_store_n(&b->action, action, __ATOMIC_RELAXED);
    __atomic_store_n(&b->flags, (u32)flags, __ATOMIC_RELAXED);
    __atomic_store_n(&b->req_seq, seq, __ATOMIC_RELEASE);  // last: the device reads the four words at once
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned k = 0;; k++) {
        if (!e->srv_launch || __atomic_load_n(&b->exited, __ATOMIC_ACQUIRE) == e->srv_launch) {
            // no server, or it exited (idle) before seeing this request: (re)start it after the
            // env's own work; it serves every request past done_seq
            if (e->srv_launch) HIPCHK(hipStreamSynchronize(e->srv_stream));
            HIPCHK(hipStreamSynchronize(e->stream));
            e->srv_launch = ++e->srv_next_launch;
            e->srv_board = board;
            srv_register(e, SrvReg{&b->req_seq, &b->op, &b->exited, &e->srv_seq, &e->srv_launch});
            k_single_server<<<1, 64, 0, e->srv_stream>>>(e->d, board, e->srv_d, e->srec_d, e->srv_seq, e->srv_launch);
            HIPCHK(hipGetLastError());
        }
        if (__atomic_load_n(&b->resp_seq, __ATOMIC_ACQUIRE) == seq) break;
        if ((k & 1023) == 1023) {  // a faulted server: the stream says so
            const hipError_t q = hipStreamQuery(e->srv_stream);
            if (q != hipSuccess && q != hipErrorNotReady) return fail(std::string("single-board server: ") + hipGetErrorString(q));
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10)) {
                (void)srv_stop(e);
                return fail("single-board server: no answer within 10 s");
            }
        }
    }
    e->srv_seq = seq;
    return 0;
}

// diagnostic: the server's segments of its last op (10 ns ticks): op, list, record copy, idle
extern "C" int gc_env_single_stamps(gc_env* e, uint32_t* out6) {
    if (!e || !out6) return fail("null argument");
    for (int k = 0; k < 6; k++) out6[k] = e->srv ? __atomic_load_n(&e->srv->stamps[k], __ATOMIC_ACQUIRE) : 0u;
    return 0;
}

extern "C" int gc_env_single_call(gc_env* e, int board, int op, int action, int flags, const gc_single_record** rec) {
    if (!e || !rec) return fail("null argument");
    if (!e->srec) return fail("call gc_env_single_setup first");
    if (board < 0 || board >= e->n) return fail("board index out of range");
    if (op < SOP_RESET || op > SOP_SYNC) return fail("op: 0 reset, 1 agent, 2 reply, 3 open, 4 sync (5 set: gc_env_single_set)");
    if (op != SOP_RESET && op != SOP_SYNC && (action < 0 || action > A_RESIGN))
        return fail("action out of range [0, 4100]");
    HIPCHK(hipSetDevice(e->device));
    if (e->d.ic.spill.ent) {  // a BLACK agent: the spill table's host checks need the stream
        if (devsrv_quiesce(e->device) || spill_before(e)) return -1;
    }
    if (srv_enabled() && !e->d.ic.spill.ent) {
        if (srv_call(e, board, op, action, flags)) return -1;
    } else {
        if (devsrv_quiesce(e->device)) return -1;
        k_single<<<1, 64, 0, e->stream>>>(e->d, board, op, action, flags, e->srec_d);
        HIPCHK(hipGetLastError());
        if (spill_after(e) || gc_env_synchronize(e)) return -1;
    }
    e->policy_ready = false;
    *rec = e->srec;
    return 0;
}

// the state setter (chess_v2.py:315-323) of one board: its pieces and the six flags; the side
// to move, move_count, done and the 3-fold window stay (k_single's SET)
extern "C" int gc_env_single_set(gc_env* e, int board, const int8_t* board64, const uint8_t* flags6,
                                 const gc_single_record** rec) {
    if (!e || !board64 || !flags6 || !rec) return fail("null argument");
    if (!e->srec) return fail("call gc_env_single_setup first");
    if (board < 0 || board >= e->n) return fail("board index out of range");
    for (int k = 0; k < 64; k++)
        if (board64[k] < -6 || board64[k] > 6) return fail("board: piece ids are -6..6");
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));  // the record is the launch's input here
    memcpy(e->srec->board, board64, 64);
    for (int k = 0; k < 4; k++) e->srec->rights[k] = flags6[k] ? 1 : 0;
    for (int k = 0; k < 2; k++) e->srec->checked[k] = flags6[4 + k] ? 1 : 0;
    if (srv_enabled() && !e->d.ic.spill.ent) {
        if (srv_call(e, board, SOP_SET, 0, 0)) return -1;
    } else {
        if (devsrv_quiesce(e->device)) return -1;
        k_single<<<1, 64, 0, e->stream>>>(e->d, board, SOP_SET, 0, 0, e->srec_d);
        HIPCHK(hipGetLastError());
        if (gc_env_synchronize(e)) return -1;
    }
    e->policy_ready = false;
    *rec = e->srec;
    return 0;
}

extern "C" int gc_env_window_boards(gc_env* e, int board, int8_t* boards, uint8_t* counts, int cap, int* n) {
    if (!e || !n || (cap > 0 && (!boards || !counts))) return fail("null argument");
    SRV_QUIESCE(e);
    if (board < 0 || board >= e->n) return fail("board index out of range");
    HIPCHK(hipSetDevice(e->device));
    int8_t* db = nullptr;
    uint8_t* dc = nullptr;
    int* dn = nullptr;
    const int c = cap > 0 ? cap : 0;
    if (dalloc(&db, (size_t)64 * (c ? c : 1)) || dalloc(&dc, c ? c : 1) || dalloc(&dn, 1)) {
        (void)hipFree(db); (void)hipFree(dc);
        return -1;
    }
    k_window_boards<<<1, 64, 0, e->stream>>>(e->d, board, db, dc, c, dn);
    hipError_t he = hipGetLastError();
    if (he == hipSuccess) he = hipMemcpyAsync(n, dn, sizeof(int), hipMemcpyDeviceToHost, e->stream);
    if (he == hipSuccess) he = hipStreamSynchronize(e->stream);
    const int k = *n < c ? *n : c;
    if (he == hipSuccess && k) he = hipMemcpy(boards, db, (size_t)64 * k, hipMemcpyDeviceToHost);
    if (he == hipSuccess && k) he = hipMemcpy(counts, dc, (size_t)k, hipMemcpyDeviceToHost);
    (void)hipFree(db); (void)hipFree(dc); (void)hipFree(dn);
    if (he != hipSuccess) return fail(std::string("window readout: ") + hipGetErrorString(he));
    return 0;
}

extern "C" int gc_env_step(gc_env* e, const uint16_t* actions, int32_t* reward, uint8_t* done, uint8_t* reason) {
    if (!e || !actions) return fail("null argument");
    SRV_QUIESCE(e);
    for (int i = 0; i < e->n; i++)
        if (actions[i] > A_RESIGN) return fail("action out of range [0, 4100] at index " + std::to_string(i));
    HIPCHK(hipSetDevice(e->device));
    if (spill_before(e)) return -1;
    HIPCHK(hipMemcpyAsync(e->d.act, actions, (size_t)2 * e->n, hipMemcpyHostToDevice, e->stream));
    launch_step<false>(e);
    HIPCHK(hipGetLastError());
    if (spill_after(e)) return -1;
    e->policy_ready = false;
    if (reward) HIPCHK(hipMemcpyAsync(reward, e->d.reward, (size_t)4 * e->n, hipMemcpyDeviceToHost, e->stream));
    if (done) HIPCHK(hipMemcpyAsync(done, e->d.done, e->n, hipMemcpyDeviceToHost, e->stream));
    if (reason) HIPCHK(hipMemcpyAsync(reason, e->d.reason, e->n, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return 0;
}

// step() with device buffers (k_env_step_api4 and its siblings): asynchronous on the env's
// stream (gc_env_get_stream); every pointer is device memory of n entries (mask: 65 rows of
// mask_stride words, word f of board i at f * mask_stride + i; obs: n*64 bytes); mask / obs /
// count / pick may be NULL.  The stride travels with each call: with n a multiple
// of a large power of two, packed rows n words apart alias on the same HBM channels, so a caller
// may pad them (gym_chess_amd.env.DeviceIO does); gc_env_step_device is the packed form.
extern "C" int gc_env_step_device2(gc_env* e, const uint16_t* d_actions, int32_t* d_reward, uint8_t* d_done,
                                   uint8_t* d_reason, uint64_t* d_mask, int8_t* d_obs, int32_t* d_count,
                                   uint16_t* d_pick, int flags, int64_t mask_stride) {
    if (!e || !d_actions || !d_reward || !d_done || !d_reason) return fail("null argument");
    SRV_QUIESCE(e);
    if (flags & ~1) return fail("flags: bit 0 = auto-reset");
    if (mask_stride != 0 && mask_stride < (int64_t)e->n) return fail("mask stride below the board count");
    HIPCHK(hipSetDevice(e->device));
    if (spill_before(e)) return -1;
    const int ar = flags & 1;
    const size_t ms = mask_stride ? (size_t)mask_stride : (size_t)e->n;  // the mask rows' stride
    if (e->rules) {  // FIDE: one lane per board
        if (e->d.opp)
            k_fenv_step_api<true><<<grid_for(e->n), BLOCK, 0, e->stream>>>(e->d, d_actions, d_reward, d_done, d_reason,
                                                                            d_mask, d_obs, d_count, d_pick, ar, ms);
        else
            k_fenv_step_api<false><<<grid_for(e->n), BLOCK, 0, e->stream>>>(e->d, d_actions, d_reward, d_done, d_reason,
                                                                             d_mask, d_obs, d_count, d_pick, ar, ms);
        HIPCHK(hipGetLastError());
        if (spill_after(e)) return -1;
        e->policy_ready = d_pick != nullptr;
        return 0;
    }
    if (!e->d.opp && e->d.ic.usable && e->d.ic.table) {
        const EnvDev& d = e->d;
        const ResetInfo r = reset_info(e);
        const int nb = (e->n + PAIR_BOARDS - 1) / PAIR_BOARDS;
        const ApiOut o = {d_reward, d_done, d_reason, d_mask, d_obs, d_count, d_pick, ms};
        if (!e->api_out) {
            if (dalloc(&e->api_out, 1)) return -1;
            e->api_host = {};
        }
        if (memcmp(&o, &e->api_host, sizeof o) != 0) {  // the caller's buffers changed
            e->api_host = o;
            HIPCHK(hipMemcpyAsync(e->api_out, &e->api_host, sizeof o, hipMemcpyHostToDevice, e->stream));
            HIPCHK(hipStreamSynchronize(e->stream));  // api_host may change again before a lazy copy ran
        }
        // (over two board-range streams, so a range's store tail could overlap the other's
        // generation: measured 47 vs 21 us per step with the paired kernel, round 3)
        k_env_step_api4<<<(nb + QUADS_WG - 1) / QUADS_WG, 4 * QUAD_BOARDS * QUADS_WG, 0, e->stream>>>(
            e->slab, d.seed, d.htab, r.racts, r.icd, d_actions, e->api_out, d.n, r.rinfo | ((u32)ar << 17));
    } else if (e->d.opp && pair_ok(e)) {  // the random opponent on the paired driver
        const EnvDev& d = e->d;
        const ResetInfo r = reset_info(e);
        const int nb = (e->n + PAIR_BOARDS - 1) / PAIR_BOARDS;
        const ApiOut o = {d_reward, d_done, d_reason, d_mask, d_obs, d_count, d_pick, ms};
        if (!e->api_out) {
            if (dalloc(&e->api_out, 1)) return -1;
            e->api_host = {};
        }
        if (memcmp(&o, &e->api_host, sizeof o) != 0) {
            e->api_host = o;
            HIPCHK(hipMemcpyAsync(e->api_out, &e->api_host, sizeof o, hipMemcpyHostToDevice, e->stream));
            HIPCHK(hipStreamSynchronize(e->stream));
        }
        const dim3 grid((nb + PAIRS_WG - 1) / PAIRS_WG), block(2 * PAIR_BOARDS * PAIRS_WG);
        const char* nq = getenv("GC_NO_QUAD_API");  // A/B and tests (read per call): api2_vs
        const bool no_quad_vs = nq && atoi(nq) != 0;
        // (a BLACK agent's resets open with the opponent's move: the openings' positions and moves
        // are cached, k_init_open_cache -- 33.9 vs 41.1 us per launch for the paired kernel,
        // tools/api_color_probe.py; through the per-piece fallback instead: 46.9)
        if (!no_quad_vs && d.agent_black && d.ic.open)  // four waves per 64 boards (k_env_step_api4_vs)
            k_env_step_api4_vs<true><<<(nb + QUADS_WG - 1) / QUADS_WG, 4 * QUAD_BOARDS * QUADS_WG, 0, e->stream>>>(
                e->slab, d.seed, d.htab, r.racts, r.icd, d_actions, e->api_out, d.n, r.rinfo | ((u32)ar << 17));
        else if (!no_quad_vs && !d.agent_black)
            k_env_step_api4_vs<false><<<(nb + QUADS_WG - 1) / QUADS_WG, 4 * QUAD_BOARDS * QUADS_WG, 0, e->stream>>>(
                e->slab, d.seed, d.htab, r.racts, r.icd, d_actions, e->api_out, d.n, r.rinfo | ((u32)ar << 17));
        else if (d.agent_black)
            k_env_step_api2_vs<true><<<grid, block, 0, e->stream>>>(e->slab, d.seed, d.htab, r.racts, r.icd, d_actions,
                                                                     e->api_out, d.n, r.rinfo | ((u32)ar << 17));
        else
            k_env_step_api2_vs<false><<<grid, block, 0, e->stream>>>(e->slab, d.seed, d.htab, r.racts, r.icd, d_actions,
                                                                      e->api_out, d.n, r.rinfo | ((u32)ar << 17));
    } else if (e->d.opp)
        k_env_step_api<true><<<grid_for(e->n), BLOCK, 0, e->stream>>>(e->d, d_actions, d_reward, d_done, d_reason,
                                                                      d_mask, d_obs, d_count, d_pick, ar, ms);
    else
        k_env_step_api<false><<<grid_for(e->n), BLOCK, 0, e->stream>>>(e->d, d_actions, d_reward, d_done, d_reason,
                                                                       d_mask, d_obs, d_count, d_pick, ar, ms);
    HIPCHK(hipGetLastError());
    if (spill_after(e)) return -1;
    e->policy_ready = d_pick != nullptr;
    return 0;
}

extern "C" int gc_env_step_device(gc_env* e, const uint16_t* d_actions, int32_t* d_reward, uint8_t* d_done,
                                  uint8_t* d_reason, uint64_t* d_mask, int8_t* d_obs, int32_t* d_count,
                                  uint16_t* d_pick, int flags) {
    return gc_env_step_device2(e, d_actions, d_reward, d_done, d_reason, d_mask, d_obs, d_count, d_pick, flags, 0);
}

extern "C" int gc_env_get_stream(gc_env* e, void** stream) {
    if (!e || !stream) return fail("null argument");
    *stream = (void*)e->stream;
    return 0;
}

// device buffers for callers without their own allocator (tests, bench): hipMalloc /
// hipFree on the env's device, and copies on its stream
extern "C" int gc_device_alloc(int device, uint64_t bytes, void** ptr) {
    if (!ptr) return fail("null argument");
    HIPCHK(hipSetDevice(device));
    HIPCHK(hipMalloc(ptr, bytes ? bytes : 1));
    return 0;
}
extern "C" int gc_device_free(int device, void* ptr) {
    HIPCHK(hipSetDevice(device));
    HIPCHK(hipFree(ptr));
    return 0;
}
extern "C" int gc_env_copy(gc_env* e, void* dst, const void* src, uint64_t bytes, int kind) {
    if (!e || !dst || !src) return fail("null argument");
    if (kind < 0 || kind > 3) return fail("kind: 0 h2h, 1 h2d, 2 d2h, 3 d2d");
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipMemcpyAsync(dst, src, bytes, (hipMemcpyKind)kind, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return 0;
}

// n plies of the paired step kernel after the work already on the env's stream: on the
// env's stream, or over the board-range streams (forked from it and joined back into it)
static int issue_plies(gc_env* e, int n) {
    if (e->n_sub <= 1) {
        for (int p = 0; p < n; p++) launch_step2(e, e->stream);
        HIPCHK(hipGetLastError());
        return 0;
    }
    const int blocks = (e->n + PAIR_BOARDS - 1) / PAIR_BOARDS;
    const int k = e->n_sub < blocks ? e->n_sub : blocks;
    // a range is a whole number of workgroups (PAIRS_WG blocks each), so no workgroup reaches
    // into the next range; only the last range is partial, and beyond it every lane is dead
    const int per = ((blocks + k - 1) / k + PAIRS_WG - 1) / PAIRS_WG * PAIRS_WG;
    HIPCHK(hipEventRecord(e->fork_ev, e->stream));
    for (int j = 0; j < k; j++) HIPCHK(hipStreamWaitEvent(e->sub[j], e->fork_ev, 0));
    for (int p = 0; p < n; p++)
        for (int j = 0; j < k; j++) {
            int b0 = j * per, nb = blocks - b0 < per ? blocks - b0 : per;
            if (nb > 0) launch_step2(e, e->sub[j], b0, nb);
        }
    HIPCHK(hipGetLastError());
    for (int j = 0; j < k; j++) {
        HIPCHK(hipEventRecord(e->sub_ev[j], e->sub[j]));
        HIPCHK(hipStreamWaitEvent(e->stream, e->sub_ev[j], 0));
    }
    return 0;
}

// device-resident random self-play: n_plies launches of the one-ply step kernel (no host
// traffic, no sync).  Outputs of the LAST ply stay in device buffers (gc_env_get_outputs).
static int step_random(gc_env* e, int n_plies);
extern "C" int gc_env_step_random(gc_env* e, int n_plies) {
    if (!e) return fail("null env");
    SRV_QUIESCE(e);
    if (!e->policy_ready) return fail("policy actions stale: call gc_env_reset or gc_env_select_random first");
    HIPCHK(hipSetDevice(e->device));
    if (spill_before(e)) return -1;
    for (int p = 0; p < n_plies;) {  // one chunk unless the env spills (spill_chunk)
        const int k = spill_chunk(e, n_plies - p);
        if (k < 0 || step_random(e, k)) return -1;
        p += k;
    }
    return spill_after(e);
}
// (a hipGraph of the plies' launches was measured slower: 11.4 vs 9.8 us per ply, round 2)
static int step_random(gc_env* e, int n_plies) {
    const bool pair = pair_ok(e);  // the paired kernel (pair_ok: all but rare opponent setups)
    int p = 0;
    if (p < n_plies) {
        if (pair) return issue_plies(e, n_plies - p);
        for (; p < n_plies; p++) {
            launch_step<true>(e);
            HIPCHK(hipGetLastError());
        }
    }
    return 0;
}

// board-range streams of gc_env_step_random (1 = the env's stream only)
extern "C" int gc_env_set_streams(gc_env* e, int k) {
    if (!e) return fail("null env");
    if (k < 1 || k > GC_MAX_SUBSTREAMS) return fail("streams must be in [1, 8]");
    HIPCHK(hipSetDevice(e->device));
    for (int j = 0; j < k; j++) {
        if (!e->sub[j]) HIPCHK(hipStreamCreateWithFlags(&e->sub[j], hipStreamNonBlocking));
        if (!e->sub_ev[j]) HIPCHK(hipEventCreateWithFlags(&e->sub_ev[j], hipEventDisableTiming));
    }
    if (!e->fork_ev) HIPCHK(hipEventCreateWithFlags(&e->fork_ev, hipEventDisableTiming));
    e->n_sub = k;
    return 0;
}

extern "C" int gc_env_paired(gc_env* e) {
    if (!e) return fail("null env");
    return pair_ok(e) ? 1 : 0;
}

// The quads take a reset board's pick from the start position's table only (Q1 reads it in
// phase 0, before the ply's outcome is known); a start position without one (> 16 own pieces,
// or more than RESET_ACTS_MAX moves) runs on the paired kernel, whose pair_ply regenerates the
// start position's move sets at a reset.
static bool use_quad(const gc_env* e) {
    static const bool no_quad = getenv("GC_NO_QUAD") != nullptr;  // A/B: the paired kernel
    return !no_quad && !e->rules && pair_opp(e) == 0 && e->d.ic.table;
}

// The occupancy filter (k_env_rollout4<true>, above) costs Q1 ~700 cycles of phase 1 and the
// ply ~3 % more cycles (tools/pstamp_probe.py); what it buys is half the ply's HBM bytes, and
// with them the clock a long launch holds under the power limit (r06h stamps: 2.27 vs 2.18 GHz
// over 1 000 plies).  Same box, always / never, the workgroups taking turns (profiles/r06_v1/
// ab_summary.txt, run_r06q): K = 20 12.86 / 13.27e9, 100 15.29 / 15.48, 300 15.73 / 15.90, 500
// 15.79 / 15.91, 700 15.91 / 15.43, 1 000 15.94 / 15.12, 2 000 16.26 / 15.62 -- so it runs for
// launches of GC_OCC_MIN_PLIES (600, the crossover) plies or more
static int occ_min_plies() {
    static const int v = getenv("GC_OCC_MIN_PLIES") ? atoi(getenv("GC_OCC_MIN_PLIES")) : 600;
    return v;
}

extern "C" int gc_env_rollout_occ_min_plies(void) { return occ_min_plies(); }

extern "C" int gc_env_rollout_waves(gc_env* e) {
    if (!e) return fail("null env");
    return pair_ok(e) ? (use_quad(e) ? 4 : 2) : 1;
}

extern "C" int gc_env_select_random(gc_env* e) {
    if (!e) return fail("null env");
    SRV_QUIESCE(e);
    HIPCHK(hipSetDevice(e->device));
    if (e->rules) k_fenv_select<<<grid_for(e->n), BLOCK, 0, e->stream>>>(e->d);
    else k_select<<<grid_for(e->n), BLOCK, 0, e->stream>>>(e->d);
    HIPCHK(hipGetLastError());
    e->policy_ready = true;
    return 0;
}

// n_plies of fused random self-play after the work already on the env's stream (no host
// sync): ROLLOUT_MAX_PLIES per launch; the per-ply trace (device memory, [n_plies][N] words,
// trace_word) when d_trace is not NULL; with `stats`, per-board stats accumulate into e->stats.
static int issue_rollout(gc_env* e, int n_plies, uint64_t* d_trace, bool stats) {
    uint64_t* const st = stats ? e->stats : nullptr;
    const bool pair = pair_ok(e);
    const EnvDev& d = e->d;
    const ResetInfo r = reset_info(e);
    const int grid = (e->n + PAIR_BOARDS * PAIRS_WG - 1) / (PAIR_BOARDS * PAIRS_WG), bs = 2 * PAIR_BOARDS * PAIRS_WG;
    for (int p0 = 0, k = 0; p0 < n_plies; p0 += k) {
        k = spill_chunk(e, n_plies - p0 < ROLLOUT_MAX_PLIES ? n_plies - p0 : ROLLOUT_MAX_PLIES);
        if (k < 0) return -1;
        u64* tr = d_trace ? reinterpret_cast<u64*>(d_trace) + (size_t)p0 * e->n : nullptr;
        const u32 ri = r.rinfo | ((u32)k << 18);
        e->done_expect = 0;
        if (pair && use_quad(e)) {
            const int qg = (e->n + QUAD_BOARDS * QUADS_WG - 1) / (QUAD_BOARDS * QUADS_WG);
            if (k >= occ_min_plies())
                k_env_rollout4<true><<<qg, 4 * QUAD_BOARDS * QUADS_WG, 0, e->stream>>>(e->slab, d.n, d.seed, d.htab,
                                                                                      sw_table(r), r.icd, ri, st, tr);
            else
                k_env_rollout4<false><<<qg, 4 * QUAD_BOARDS * QUADS_WG, 0, e->stream>>>(e->slab, d.n, d.seed, d.htab,
                                                                                       sw_table(r), r.icd, ri, st, tr);
            e->done_expect = ++e->done_issued;
        } else if (pair) {
            switch (e->rules ? 3 : pair_opp(e)) {
                case 3: k_env_rollout2<true><<<grid, bs, 0, e->stream>>>(e->slab, d.n, d.seed, d.htab, r.racts, r.icd, ri, st, tr); break;
                case 0: k_env_rollout2<false><<<grid, bs, 0, e->stream>>>(e->slab, d.n, d.seed, d.htab, sw_table(r), r.icd, ri, st, tr); break;
                case 1: k_env_rollout2<false, 1><<<grid, bs, 0, e->stream>>>(e->slab, d.n, d.seed, d.htab, sw_table(r), r.icd, ri, st, tr); break;
                default: k_env_rollout2<false, 2><<<grid, bs, 0, e->stream>>>(e->slab, d.n, d.seed, d.htab, sw_table(r), r.icd, ri, st, tr); break;
            }
        } else if (e->rules) {  // FIDE with the random opponent
            k_fenv_rollout<true><<<grid_for(e->n), BLOCK, 0, e->stream>>>(e->d, k, tr, st);
        } else if (e->d.opp) {
            k_env_rollout<true><<<grid_for(e->n), BLOCK, 0, e->stream>>>(e->d, k, tr, st);
        } else {
            k_env_rollout<false><<<grid_for(e->n), BLOCK, 0, e->stream>>>(e->d, k, tr, st);
        }
        hipError_t le = hipGetLastError();
        if (le != hipSuccess) return fail(std::string("rollout launch: ") + hipGetErrorString(le));
    }
    return 0;
}

extern "C" int gc_env_rollout(gc_env* e, int n_plies, int16_t* tr_action, int16_t* tr_reward, uint8_t* tr_done,
                              uint8_t* tr_reason, uint64_t* stats8) {
    if (!e) return fail("null env");
    SRV_QUIESCE(e);
    if (n_plies < 0) return fail("n_plies must be >= 0");
    if (!e->policy_ready) return fail("policy actions stale: call gc_env_reset or gc_env_select_random first");
    HIPCHK(hipSetDevice(e->device));
    const bool trace = tr_action || tr_reward || tr_done || tr_reason;
    const size_t cnt = (size_t)n_plies * e->n;
    u64* dt = nullptr;
    if (trace && cnt && dalloc(&dt, cnt)) return -1;
    if (spill_before(e)) { (void)hipFree(dt); return -1; }
    HIPCHK(hipMemsetAsync(e->stats, 0, (size_t)64 * e->n, e->stream));
    if (issue_rollout(e, n_plies, dt, true) || spill_after(e)) { (void)hipFree(dt); return -1; }
    if (trace && cnt) {
        std::vector<u64> h(cnt);
        hipError_t ce = hipMemcpyAsync(h.data(), dt, cnt * 8, hipMemcpyDeviceToHost, e->stream);
        if (ce == hipSuccess) ce = hipStreamSynchronize(e->stream);
        (void)hipFree(dt);
        if (ce != hipSuccess) return fail(std::string("rollout trace: ") + hipGetErrorString(ce));
        for (size_t t = 0; t < cnt; t++) {
            const u64 w = h[t];
            if (tr_action) tr_action[t] = (int16_t)(uint16_t)w;
            if (tr_reward) tr_reward[t] = (int16_t)(uint16_t)(w >> 16);
            if (tr_done) tr_done[t] = (uint8_t)(w >> 32);
            if (tr_reason) tr_reason[t] = (uint8_t)(w >> 40);
        }
    }
    if (stats8) {
        uint64_t* sums = e->stats + (size_t)8 * e->n;
        HIPCHK(hipMemsetAsync(sums, 0, 64, e->stream));
        k_sum_stats<<<grid_for(e->n), BLOCK, 0, e->stream>>>(e->stats, e->n, reinterpret_cast<unsigned long long*>(sums));
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(stats8, sums, 64, hipMemcpyDeviceToHost, e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));
    }
    return 0;
}

// n_plies env.step() calls of every board under the random self-play policy in one launch
// (per ROLLOUT_MAX_PLIES), asynchronous on the env's stream; each ply's outputs land in the
// device trace [n_plies][N] (trace_word) when d_trace is not NULL.  State, windows, counters
// and the last ply's outputs afterwards are those of n_plies gc_env_step_random plies.
// ev_begin / ev_end: event slots (gc_env_record_event) recorded on the env's stream right
// before / after the launches, -1 = none (one C-ABI call brackets the timed work).
extern "C" int gc_env_rollout_device(gc_env* e, int n_plies, uint64_t* d_trace, int ev_begin, int ev_end) {
    if (!e) return fail("null env");
    SRV_QUIESCE(e);
    if (n_plies < 0) return fail("n_plies must be >= 0");
    if (ev_begin < -1 || ev_begin >= 8 || ev_end < -1 || ev_end >= 8) return fail("event slots: -1 or 0..7");
    if (!e->policy_ready) return fail("policy actions stale: call gc_env_reset or gc_env_select_random first");
    HIPCHK(hipSetDevice(e->device));
    if (spill_before(e)) return -1;
    // marker events around the launches (r03 probe: timing the launches by hipExtLaunchKernel's
    // own start / stop events cost ~8 us more host time per call at K = 20 -- tools/short_probe.py)
    if (ev_begin >= 0) HIPCHK(hipEventRecord(e->ev[ev_begin], e->stream));
    if (issue_rollout(e, n_plies, d_trace, false)) return -1;
    if (ev_end >= 0) HIPCHK(hipEventRecord(e->ev[ev_end], e->stream));
    return spill_after(e);
}

extern "C" int gc_env_get_outputs(gc_env* e, int32_t* reward, uint8_t* done, uint8_t* reason, uint16_t* next_action,
                                  uint32_t* nsteps) {
    if (!e) return fail("null env");
    SRV_QUIESCE(e);
    HIPCHK(hipSetDevice(e->device));
    if (reward) HIPCHK(hipMemcpyAsync(reward, e->d.reward, (size_t)4 * e->n, hipMemcpyDeviceToHost, e->stream));
    if (done) HIPCHK(hipMemcpyAsync(done, e->d.done, e->n, hipMemcpyDeviceToHost, e->stream));
    if (reason) HIPCHK(hipMemcpyAsync(reason, e->d.reason, e->n, hipMemcpyDeviceToHost, e->stream));
    if (next_action) HIPCHK(hipMemcpyAsync(next_action, e->d.act, (size_t)2 * e->n, hipMemcpyDeviceToHost, e->stream));
    if (nsteps) HIPCHK(hipMemcpyAsync(nsteps, e->d.nsteps, (size_t)4 * e->n, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return 0;
}

extern "C" int gc_env_get_states(gc_env* e, int8_t* boards, uint8_t* meta) {
    if (!e) return fail("null env");
    SRV_QUIESCE(e);
    HIPCHK(hipSetDevice(e->device));
    k_export<<<grid_for(e->n), BLOCK, 0, e->stream>>>(e->d.st, e->mbox, e->m8);
    HIPCHK(hipGetLastError());
    if (boards) HIPCHK(hipMemcpyAsync(boards, e->mbox, (size_t)64 * e->n, hipMemcpyDeviceToHost, e->stream));
    if (meta) HIPCHK(hipMemcpyAsync(meta, e->m8, (size_t)8 * e->n, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return 0;
}

// set states (FEN/dict ingest). meta8[7] = move_count; repetition windows are cleared.
extern "C" int gc_env_set_states(gc_env* e, const int8_t* boards, const uint8_t* meta) {
    if (!e || !boards || !meta) return fail("null argument");
    SRV_QUIESCE(e);
    if (check_boards(e->n, boards)) return -1;
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipMemcpyAsync(e->mbox, boards, (size_t)64 * e->n, hipMemcpyHostToDevice, e->stream));
    HIPCHK(hipMemcpyAsync(e->m8, meta, (size_t)8 * e->n, hipMemcpyHostToDevice, e->stream));
    if (e->rules) k_fenv_import<<<grid_for(e->n), BLOCK, 0, e->stream>>>(e->mbox, e->m8, nullptr, e->d);
    else k_env_import<<<grid_for(e->n), BLOCK, 0, e->stream>>>(e->mbox, e->m8, e->d, 0);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(e->stream));
    if (spill_windows_cleared(e)) return -1;
    e->policy_ready = false;
    return 0;
}

// ----------------------------------------------------------------------------- FEN
// Forsyth-Edwards ingest/export for the reference's state: piece
// placement rank 8 first (= board row 0, lib.rs:41-50), side to move, castling -> the four
// *_castle_is_possible flags; en passant and the half-move clock do not exist under the
// reference's rules and are ignored; the full-move number n maps to move_count = n - 1
// (chess_v2.py:291-292 counts completed full moves).  Host code, no GPU needed.
static const char* FEN_PIECES = ".KQRBNP";

extern "C" int gc_fen_to_state(const char* fen, int8_t* board, uint8_t* meta) {
    return gc_fen_to_state_rules(fen, board, meta, 0);
}

// rules 1 (FIDE): the en-passant field is parsed (it must be on the rank the side to move
// captures onto) and meta8[7] = its file + 1 (0 = "-"), the engine's FIDE convention
extern "C" int gc_fen_to_state_rules(const char* fen, int8_t* board, uint8_t* meta, int rules) {
    if (!fen || !board || !meta) return fail("null argument");
    int8_t b[64] = {0};
    const char* p = fen;
    while (*p == ' ') p++;
    int row = 0, col = 0;
    for (; *p && *p != ' '; p++) {
        char c = *p;
        if (c == '/') {
            if (col != 8 || row >= 7) return fail(std::string("FEN: bad rank at '") + fen + "'");
            row++;
            col = 0;
        } else if (c >= '1' && c <= '8') {
            col += c - '0';
            if (col > 8) return fail(std::string("FEN: rank overflow in '") + fen + "'");
        } else {
            const char* q = strchr(FEN_PIECES + 1, c >= 'a' ? c - 32 : c);
            if (!q || c == '.' || col >= 8) return fail(std::string("FEN: bad piece '") + c + "' in '" + fen + "'");
            int id = (int)(q - FEN_PIECES);
            b[row * 8 + col++] = (int8_t)(c >= 'a' ? -id : id);
        }
    }
    if (row != 7 || col != 8) return fail(std::string("FEN: placement must have 8 full ranks: '") + fen + "'");
    uint8_t m[8] = {1, 0, 0, 0, 0, 0, 0, 0};
    while (*p == ' ') p++;
    if (*p) {
        if (*p == 'b') m[0] = 0;
        else if (*p != 'w') return fail(std::string("FEN: side to move must be w or b: '") + fen + "'");
        p++;
        while (*p == ' ') p++;
        for (; *p && *p != ' '; p++) {
            switch (*p) {
                case 'K': m[1] = 1; break;
                case 'Q': m[2] = 1; break;
                case 'k': m[3] = 1; break;
                case 'q': m[4] = 1; break;
                case '-': break;
                default: return fail(std::string("FEN: bad castling field in '") + fen + "'");
            }
        }
        // reference rules: en passant and half-move clock ignored, full-move number ->
        // move_count; FIDE: en passant -> meta8[7]
        int field = 0;
        long full = 1;
        int epf = -1;
        while (*p) {
            while (*p == ' ') p++;
            if (!*p) break;
            const char* st = p;
            while (*p && *p != ' ') p++;
            ++field;
            if (field == 1 && rules && !(p - st == 1 && *st == '-')) {
                int want = m[0] ? '6' : '3';
                if (p - st != 2 || st[0] < 'a' || st[0] > 'h' || st[1] != want)
                    return fail(std::string("FEN: bad en-passant field in '") + fen + "'");
                epf = st[0] - 'a';
            }
            if (field == 3) {
                char* end = nullptr;
                full = strtol(st, &end, 10);
                if (end != p || full < 1) return fail(std::string("FEN: bad full-move number in '") + fen + "'");
            }
        }
        long mc = full - 1;
        m[7] = rules ? (uint8_t)(epf + 1) : (uint8_t)(mc > 255 ? 255 : mc);
    }
    memcpy(board, b, 64);
    memcpy(meta, m, 8);
    return 0;
}

extern "C" int gc_state_to_fen(const int8_t* board, const uint8_t* meta, char* out, int cap) {
    return gc_state_to_fen_rules(board, meta, out, cap, 0);
}

extern "C" int gc_state_to_fen_rules(const int8_t* board, const uint8_t* meta, char* out, int cap, int rules) {
    if (!board || !meta || !out) return fail("null argument");
    if (check_boards(1, board)) return -1;
    std::string f;
    for (int r = 0; r < 8; r++) {
        int gap = 0;
        for (int c = 0; c < 8; c++) {
            int v = board[r * 8 + c];
            if (!v) { gap++; continue; }
            if (gap) { f += (char)('0' + gap); gap = 0; }
            char ch = FEN_PIECES[v < 0 ? -v : v];
            f += v < 0 ? (char)(ch + 32) : ch;
        }
        if (gap) f += (char)('0' + gap);
        if (r < 7) f += '/';
    }
    f += meta[0] ? " w " : " b ";
    std::string cs;
    if (meta[1]) cs += 'K';
    if (meta[2]) cs += 'Q';
    if (meta[3]) cs += 'k';
    if (meta[4]) cs += 'q';
    f += cs.empty() ? "-" : cs;
    if (rules) {
        f += " ";
        if (meta[7]) { f += (char)('a' + ((meta[7] - 1) & 7)); f += meta[0] ? '6' : '3'; }
        else f += "-";
        f += " 0 1";
    } else {
        f += " - 0 " + std::to_string((int)meta[7] + 1);
    }
    if ((int)f.size() + 1 > cap) return fail("FEN output buffer too small");
    memcpy(out, f.c_str(), f.size() + 1);
    return 0;
}

// FEN ingest for the whole env: boards[i] := fens[i], check flags from update_state,
// repetition windows cleared (like gc_env_set_states)
extern "C" int gc_env_set_fens(gc_env* e, const char* const* fens) {
    if (!e || !fens) return fail("null argument");
    SRV_QUIESCE(e);
    std::vector<int8_t> b((size_t)64 * e->n), ep(e->n, -1);
    std::vector<uint8_t> m((size_t)8 * e->n);
    for (int i = 0; i < e->n; i++) {
        uint8_t* mi = m.data() + 8 * (size_t)i;
        if (gc_fen_to_state_rules(fens[i], b.data() + 64 * (size_t)i, mi, e->rules))
            return fail("board " + std::to_string(i) + ": " + g_err);
        if (e->rules) {  // meta8[7] carried the en-passant file: the env keeps move_count 0
            ep[i] = (int8_t)(mi[7] ? mi[7] - 1 : -1);
            mi[7] = 0;
        }
    }
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipMemcpyAsync(e->mbox, b.data(), b.size(), hipMemcpyHostToDevice, e->stream));
    HIPCHK(hipMemcpyAsync(e->m8, m.data(), m.size(), hipMemcpyHostToDevice, e->stream));
    if (e->rules) {
        if (!e->ep && dalloc(&e->ep, e->n)) return -1;
        HIPCHK(hipMemcpyAsync(e->ep, ep.data(), e->n, hipMemcpyHostToDevice, e->stream));
        k_fenv_import<<<grid_for(e->n), BLOCK, 0, e->stream>>>(e->mbox, e->m8, e->ep, e->d);
    } else {
        k_env_import<<<grid_for(e->n), BLOCK, 0, e->stream>>>(e->mbox, e->m8, e->d, 1);
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(e->stream));
    e->policy_ready = false;
    return 0;
}

extern "C" int gc_env_legal_moves(gc_env* e, uint16_t* moves, int cap, int32_t* counts) {
    if (!e || !moves || !counts) return fail("null argument");
    SRV_QUIESCE(e);
    if (cap <= 0) return fail("cap must be > 0");
    HIPCHK(hipSetDevice(e->device));
    if (cap > e->list_cap) {
        if (e->list) (void)hipFree(e->list);
        e->list = nullptr;
        e->list_cap = 0;
        if (dalloc(&e->list, (size_t)cap * e->n)) return -1;
        e->list_cap = cap;
    }
    if (e->rules) k_flist<<<grid_for(e->n), BLOCK, 0, e->stream>>>(e->d.st, 0, cap, e->list, e->counts);
    else k_list<<<grid_for(e->n), BLOCK, 0, e->stream>>>(e->d.st, 0, cap, e->list, e->counts);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(moves, e->list, (size_t)2 * cap * e->n, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipMemcpyAsync(counts, e->counts, (size_t)4 * e->n, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return 0;
}

extern "C" int gc_env_legal_mask(gc_env* e, uint64_t* mask, int32_t* counts) {
    if (!e || !mask) return fail("null argument");
    SRV_QUIESCE(e);
    HIPCHK(hipSetDevice(e->device));
    if (!e->lmask && dalloc(&e->lmask, (size_t)65 * e->n)) return -1;
    if (e->rules) k_fmask<<<grid_for(e->n), BLOCK, 0, e->stream>>>(e->d.st, e->lmask, e->counts);
    else k_mask<<<grid_for(e->n), BLOCK, 0, e->stream>>>(e->d.st, e->lmask, e->counts);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(mask, e->lmask, (size_t)8 * 65 * e->n, hipMemcpyDeviceToHost, e->stream));
    if (counts) HIPCHK(hipMemcpyAsync(counts, e->counts, (size_t)4 * e->n, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return 0;
}

// Wait for the env's stream.  Spin on hipStreamQuery first (bounded): a blocking
// hipStreamSynchronize can sleep on the completion interrupt and pays its wake-up on every
// short wait; after GC_SPIN_US (default 20 000 us) of spinning it blocks.
extern "C" int gc_env_synchronize(gc_env* e) {
    if (!e) return fail("null env");
    HIPCHK(hipSetDevice(e->device));
    static const long spin_us = getenv("GC_SPIN_US") ? atol(getenv("GC_SPIN_US")) : 20000;
    if (spin_us > 0) {
        const auto t0 = std::chrono::steady_clock::now();
        for (;;) {
            const hipError_t q = hipStreamQuery(e->stream);
            if (q == hipSuccess) return 0;
            if (q != hipErrorNotReady) return fail(std::string("stream: ") + hipGetErrorString(q));
            if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us)) break;
        }
    }
    HIPCHK(hipStreamSynchronize(e->stream));
    return 0;
}

// Wait for the work of the last gc_env_rollout_device call: when it ended with a quad launch,
// until that launch's completion word reaches host memory (every workgroup's stores done),
// else until the stream is idle.  Work enqueued after the launch (an event record) may still
// be pending; reads through the env's stream stay ordered after it.  Spins with a stream
// query now and then, so a word that never comes cannot hang the caller.
extern "C" int gc_env_wait_rollout(gc_env* e) {
    if (!e) return fail("null env");
    if (!e->done_expect || !e->done_host) return gc_env_synchronize(e);
    const u32 want = e->done_expect;
    for (unsigned k = 0;; k++) {
        if ((int)(__atomic_load_n(e->done_host, __ATOMIC_ACQUIRE) - want) >= 0) return 0;
        if ((k & 255) == 255) {
            const hipError_t q = hipStreamQuery(e->stream);
            if (q == hipSuccess) return 0;
            if (q != hipErrorNotReady) return fail(std::string("stream: ") + hipGetErrorString(q));
        }
    }
}

extern "C" int gc_env_record_event(gc_env* e, int slot) {
    if (!e || slot < 0 || slot >= 8) return fail("bad env or event slot");
    HIPCHK(hipEventRecord(e->ev[slot], e->stream));
    return 0;
}

extern "C" int gc_env_elapsed_ms(gc_env* e, int a, int b, float* ms) {
    if (!e || !ms || a < 0 || a >= 8 || b < 0 || b >= 8) return fail("bad argument");
    HIPCHK(hipEventSynchronize(e->ev[b]));
    HIPCHK(hipEventElapsedTime(ms, e->ev[a], e->ev[b]));
    return 0;
}

// sum over boards of the repetition-window length (bytes accounting in bench.py)
__global__ void k_window_sum(SoA st, unsigned long long* out) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long v = i < st.n ? (unsigned long long)hl_of(st.meta[i]) : 0ull;
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(out, v);
}

extern "C" int gc_env_window_sum(gc_env* e, uint64_t* sum) {
    if (!e || !sum) return fail("null argument");
    SRV_QUIESCE(e);
    HIPCHK(hipSetDevice(e->device));
    unsigned long long* d = nullptr;
    if (dalloc(&d, 1)) return -1;
    HIPCHK(hipMemsetAsync(d, 0, 8, e->stream));
    k_window_sum<<<grid_for(e->n), BLOCK, 0, e->stream>>>(e->d.st, d);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(sum, d, 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    (void)hipFree(d);
    return 0;
}

#ifdef GC_PSTAMPS
// per wave (global wave index = block * waves per block + wave): the 8 segment cycle sums of
// one fused launch of n_plies (reference rules, opponent "none"), then 4 s_memrealtime stamps:
// wave start, entry loads done, first ply done, last ply done
extern "C" int gc_debug_pstamps(gc_env* e, int n_plies, uint64_t* out /* waves * 12 */) {
    unsigned long long* d = nullptr;
    // waves of the fused launch: pairs (2 per 64 boards) or quads (4 per 64 boards)
    const size_t waves = use_quad(e) ? (size_t)((e->n + QUAD_BOARDS * QUADS_WG - 1) / (QUAD_BOARDS * QUADS_WG)) * 4 * QUADS_WG
                                     : (size_t)((e->n + PAIR_BOARDS * PAIRS_WG - 1) / (PAIR_BOARDS * PAIRS_WG)) * 2 * PAIRS_WG;
    if (dalloc(&d, waves * 12)) return -1;
    HIPCHK(hipMemsetAsync(d, 0, waves * 96, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_pst_out), &d, sizeof(d)));
    if (issue_rollout(e, n_plies, nullptr, false)) return -1;
    HIPCHK(hipMemcpyAsync(out, d, waves * 96, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    unsigned long long* z = nullptr;
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_pst_out), &z, sizeof(z)));
    (void)hipFree(d);
    return 0;
}
#endif

#ifdef GC_PSTAMPS
// the quad API step's per-wave stamps (tools/api_pstamp_probe.py): buffer on (`on` != 0, sized
// for the env's k_env_step_api4 waves, zeroed) or copied out and off
static unsigned long long* g_api_pst = nullptr;
extern "C" int gc_debug_api_pstamps(gc_env* e, int on, uint64_t* out /* waves * 12 */) {
    const size_t waves = (size_t)((e->n + QUAD_BOARDS * QUADS_WG - 1) / (QUAD_BOARDS * QUADS_WG)) * 4 * QUADS_WG;
    HIPCHK(hipStreamSynchronize(e->stream));
    if (on) {
        if (!g_api_pst && dalloc(&g_api_pst, waves * 12)) return -1;
        HIPCHK(hipMemset(g_api_pst, 0, waves * 96));
        HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_pst_out), &g_api_pst, sizeof(g_api_pst)));
        return 0;
    }
    if (g_api_pst && out) HIPCHK(hipMemcpy(out, g_api_pst, waves * 96, hipMemcpyDeviceToHost));
    unsigned long long* z = nullptr;
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_pst_out), &z, sizeof(z)));
    return 0;
}
#endif

#ifdef GC_STAMPS
extern "C" int gc_debug_stamps(gc_env* e, int n_plies, uint64_t* out /* (n/64)*8 */) {
    unsigned long long* d = nullptr;
    size_t cnt = (size_t)((e->n + 63) / 64) * 16;  // per wave: 8 stamps (the paired kernel has 2 waves / 64 boards)
    if (dalloc(&d, cnt)) return -1;
    HIPCHK(hipMemsetAsync(d, 0, cnt * 8, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_out), &d, sizeof(d)));
    for (int p = 0; p < n_plies; p++) {
        launch_step2(e, e->stream);
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(out, d, cnt * 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    unsigned long long* z = nullptr;
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_out), &z, sizeof(z)));
    (void)hipFree(d);
    return 0;
}
#endif

// en passant of the FIDE-rules env (gc_fide.h keeps it in meta bits 25..28; the env's
// meta8[7] is move_count, so it travels beside the state arrays)
__global__ void k_get_ep(SoA st, int8_t* __restrict__ files) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= st.n) return;
    u32 m = st.meta[i];
    files[i] = (m & gcf::M_EP) ? (int8_t)((m & gcf::M_EP_MASK) >> gcf::M_EP_SHIFT) : (int8_t)-1;
}
__global__ void k_set_ep(SoA st, const int8_t* __restrict__ files) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= st.n) return;
    st.meta[i] = gcf::with_ep(st.meta[i], files[i] < 0 ? -1 : (int)files[i]);
}

extern "C" int gc_env_get_en_passant(gc_env* e, int8_t* files) {
    if (!e || !files) return fail("null argument");
    HIPCHK(hipSetDevice(e->device));
    if (!e->ep && dalloc(&e->ep, e->n)) return -1;
    k_get_ep<<<grid_for(e->n), BLOCK, 0, e->stream>>>(e->d.st, e->ep);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(files, e->ep, e->n, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return 0;
}

extern "C" int gc_env_set_en_passant(gc_env* e, const int8_t* files) {
    if (!e || !files) return fail("null argument");
    for (int i = 0; i < e->n; i++) {
        if (files[i] > 7) return fail("en-passant file out of range at index " + std::to_string(i));
        if (files[i] >= 0 && !e->rules) return fail("en passant exists only under rules=fide (Q3: the reference has none)");
    }
    HIPCHK(hipSetDevice(e->device));
    if (!e->ep && dalloc(&e->ep, e->n)) return -1;
    HIPCHK(hipMemcpyAsync(e->ep, files, e->n, hipMemcpyHostToDevice, e->stream));
    k_set_ep<<<grid_for(e->n), BLOCK, 0, e->stream>>>(e->d.st, e->ep);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(e->stream));
    e->policy_ready = false;
    return 0;
}

// ----------------------------------------------------------------------------- checkpoint
// Bit-exact save / restore of a whole env (SURVEY.md §5 "save/load = memcpy of state +
// repetition history"; the reference keeps its history in ChessEnvV2.saved_boards,
// chess_v2.py:192, 404-407, beside the state dict, 301-323).  Blob layout (version 2):
//   CkptHeader | slab (Slab::BYTES_PER_BOARD * n: bitboards, meta, window generation, Philox
//   draw counter, step counter, last outputs, next action) | spill counts u32[n] (live spill
//   entries per board, zero unless a BLACK agent's window spilled) | the live window-table
//   entries, board by board (hl_of(meta[i]) entries of 8 u64: header {tag | count << 56}, 7
//   bitboards) | the live spill entries, board by board (8 u64: count, 7 bitboards).
// Only live entries travel: restoring re-inserts them under a fresh generation, so a restored
// board answers every later probe exactly as before (same boards, same counts; slot positions
// may differ, which no result depends on).  The header pins the slab's field layout
// (CKPT_LAYOUT); a blob whose windows do not fit the env's tables is refused before anything
// of the env changes.
struct CkptHeader {
    char magic[8];  // "GCCKPT2"
    uint32_t version, n, rules, opp, agent_black, policy_ready;
    uint64_t seed;
    uint64_t init[NBB];  // the env's initial board (resets land on it)
    uint64_t entries;        // window-table entries
    uint64_t spill_entries;  // spill-table entries
    uint64_t layout;         // CKPT_LAYOUT of the writer
};
static const char CKPT_MAGIC[8] = {'G', 'C', 'C', 'K', 'P', 'T', '2', 0};
// the slab's size and field offsets per board (a writer with another layout is refused)
static constexpr uint64_t CKPT_LAYOUT = (uint64_t)Slab::BYTES_PER_BOARD | (56ull << 8) | (60ull << 16) | (64ull << 24) |
                                        (68ull << 32) | (72ull << 40) | (76ull << 48) | (78ull << 56);
static_assert(Slab::BYTES_PER_BOARD == 80, "update CKPT_LAYOUT with the slab");

__global__ void k_hl_of(const u32* __restrict__ meta, int n, uint32_t* __restrict__ hl) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) hl[i] = hl_of(meta[i]);
}

// the live entries (generation == hgen[i]) of board i, in table order, at out[offs[i]..]
__global__ void k_ckpt_pack(const u64* __restrict__ htab, const u32* __restrict__ hgen, const u32* __restrict__ meta,
                            int n, int nb, const uint32_t* __restrict__ offs, u64* __restrict__ out,
                            uint32_t* __restrict__ bad) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    DevHist h{const_cast<u64*>(htab), const_cast<u32*>(hgen), hgen[i], i, nb};
    const u32 g = h.gen(), hl = hl_of(meta[i]);
    u32 k = 0;
    u64* o = out + (size_t)offs[i] * 8;
    for (int pos = 0; pos < (1 << nb); pos++) {
        const u64* e = htab + h.entry(pos) * 8;
        u64 hdr = e[0];
        if ((u32)hdr != g) continue;
        if (k < hl) {
            u64* d = o + (size_t)k * 8;
            d[0] = hdr & ~0xFFFFFFFFull;  // tag | count; the generation is re-issued on restore
#pragma unroll
            for (int j = 1; j < 8; j++) d[j] = e[j];
        }
        k++;
    }
    if (k != hl) atomicOr(bad, 1u);
}

// live spill entries per board (cnt zeroed by the caller); with out: packed at
// out[offs[owner] + fill[owner]++] as {count, 7 bitboards}
__global__ void k_spill_collect(const u64* __restrict__ ent, u32 mask, const u32* __restrict__ hgen,
                                uint32_t* __restrict__ cnt, const uint32_t* __restrict__ offs, u64* __restrict__ out) {
    const size_t slot = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (slot > mask) return;
    const u64* e = ent + slot * 8;
    const u64 hdr = e[0];
    const u32 o1 = sp_owner1(hdr);
    if (o1 == 0 || sp_gen(hdr) != hgen[o1 - 1]) return;
    const u32 k = atomicAdd(cnt + (o1 - 1), 1u);
    if (!out) return;
    u64* d = out + ((size_t)offs[o1 - 1] + k) * 8;
    d[0] = sp_cnt(hdr);
#pragma unroll
    for (int j = 1; j < 8; j++) d[j] = e[j];
}

// fresh generation per board: above both the live table's and the saved one, so no entry of
// the live table can pass for a restored one
__global__ void k_ckpt_gen(const u32* __restrict__ live_hgen, const u32* __restrict__ saved_hgen, int n,
                           uint32_t* __restrict__ gnew) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) gnew[i] = (live_hgen[i] > saved_hgen[i] ? live_hgen[i] : saved_hgen[i]) + 1u;
}

// refuse a blob whose windows do not fit the env's tables (before the env changes): a window
// longer than hist_cap, or spill entries without a full table or without a spill table
__global__ void k_ckpt_check(const u32* __restrict__ meta, const uint32_t* __restrict__ scnt, int n, int nb, int spill,
                             uint32_t* __restrict__ bad) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int hl = (int)hl_of(meta[i]);
    if (hl > hist_cap(nb)) atomicOr(bad, 1u);
    if (scnt[i] && (!spill || hl < hist_cap(nb))) atomicOr(bad, 2u);
}

// board i takes generation gnew[i] and its saved entries are inserted by the probe rule of
// rep_commit (gc_env.h): home slot = key & (HTAB-1), linear probing; its spill entries by
// spill_insert's
__global__ void k_ckpt_unpack(u64* __restrict__ htab, u32* __restrict__ hgen, const u32* __restrict__ meta, int n,
                              int nb, const uint32_t* __restrict__ gnew, const uint32_t* __restrict__ offs,
                              const u64* __restrict__ in, SpillTab sp, const uint32_t* __restrict__ scnt,
                              const uint32_t* __restrict__ soffs, const u64* __restrict__ sin, uint32_t* __restrict__ bad) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const u32 g = gnew[i];
    hgen[i] = g;
    DevHist h{htab, hgen, g, i, nb};
    h.sp = sp;
    const u32 hl = hl_of(meta[i]);
    const int size = 1 << nb;
    for (u32 k = 0; k < hl; k++) {
        const u64* e = in + ((size_t)offs[i] + k) * 8;
        Pos b = {e[1], e[2], e[3], e[4], e[5], e[6], e[7], 0};
        u32 key = board_key(b);
        u32 pos = key & (size - 1), tag = key >> nb;
        int probe = 0;
        while ((u32)htab[h.entry((int)pos) * 8] == g && probe < size) { pos = (pos + 1) & (size - 1); probe++; }
        if (probe == size) { atomicOr(bad, 2u); return; }
        u64* d = htab + h.entry((int)pos) * 8;
        d[0] = (u64)g | ((u64)tag << 32) | (e[0] & (0xFFull << 56));
#pragma unroll
        for (int j = 1; j < 8; j++) d[j] = e[j];
    }
    for (u32 k = 0; k < (scnt ? scnt[i] : 0u); k++) {
        const u64* e = sin + ((size_t)soffs[i] + k) * 8;
        Pos b = {e[1], e[2], e[3], e[4], e[5], e[6], e[7], 0};
        if (!spill_insert(h, b, board_key(b))) { atomicOr(bad, 4u); return; }
        u32 t = sp_home(board_key(b), (u32)i, sp.mask);  // the entry just inserted: set its count
        for (int probe = 0; probe < SPILL_PROBES; probe++, t = (t + 1) & sp.mask) {
            const u64 x = h.sp_hdr(t);
            if (sp_owner1(x) == (u32)i + 1 && sp_gen(x) == g && h.sp_same(t, b)) {
                h.sp_set_hdr(t, sp_make((u32)i, g, (u32)e[0]));
                break;
            }
        }
    }
}

// exclusive scan of v (n entries) -> offs; returns the total
static int scan_u32(gc_env* e, const uint32_t* v, uint32_t* offs, int n, uint64_t* total) {
    size_t tb = 0;
    void* tmp = nullptr;
    hipError_t he = hipcub::DeviceScan::ExclusiveSum(nullptr, tb, v, offs, n, e->stream);
    if (he == hipSuccess && dalloc((char**)&tmp, tb ? tb : 1)) return -1;
    if (he == hipSuccess) he = hipcub::DeviceScan::ExclusiveSum(tmp, tb, v, offs, n, e->stream);
    uint32_t lo = 0, lc = 0;
    if (he == hipSuccess) he = hipMemcpyAsync(&lo, offs + n - 1, 4, hipMemcpyDeviceToHost, e->stream);
    if (he == hipSuccess) he = hipMemcpyAsync(&lc, v + n - 1, 4, hipMemcpyDeviceToHost, e->stream);
    if (he == hipSuccess) he = hipStreamSynchronize(e->stream);
    (void)hipFree(tmp);
    if (he != hipSuccess) return fail(std::string("checkpoint scan: ") + hipGetErrorString(he));
    *total = (uint64_t)lo + lc;
    return 0;
}

// exclusive scan of the window lengths of `meta` (the saved or live slab's) -> offs; returns
// the total entry count
static int ckpt_offsets(gc_env* e, const u32* meta, uint32_t* hl, uint32_t* offs, uint64_t* total) {
    k_hl_of<<<grid_for(e->n), BLOCK, 0, e->stream>>>(meta, e->n, hl);
    return scan_u32(e, hl, offs, e->n, total);
}

// live spill entries per board (scnt) and their offsets (soffs); total
static int spill_offsets(gc_env* e, uint32_t* scnt, uint32_t* soffs, uint64_t* total) {
    HIPCHK(hipMemsetAsync(scnt, 0, (size_t)4 * e->n, e->stream));
    const SpillTab& sp = e->d.ic.spill;
    if (sp.ent) {
        const size_t slots = (size_t)sp.mask + 1;
        k_spill_collect<<<(unsigned)((slots + BLOCK - 1) / BLOCK), BLOCK, 0, e->stream>>>(sp.ent, sp.mask, e->d.hgen, scnt,
                                                                                          nullptr, nullptr);
        HIPCHK(hipGetLastError());
    }
    return scan_u32(e, scnt, soffs, e->n, total);
}

static size_t ckpt_bytes(int n, uint64_t entries, uint64_t spill_entries) {
    return sizeof(CkptHeader) + (Slab::BYTES_PER_BOARD + 4) * (size_t)n + 64 * (size_t)(entries + spill_entries);
}

extern "C" int gc_env_checkpoint_bytes(gc_env* e, uint64_t* bytes) {
    if (!e || !bytes) return fail("null argument");
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    uint32_t *hl = nullptr, *offs = nullptr;
    if (dalloc(&hl, e->n) || dalloc(&offs, e->n)) { (void)hipFree(hl); return -1; }
    uint64_t total = 0, stotal = 0;
    int rc = ckpt_offsets(e, e->meta, hl, offs, &total);
    if (!rc) rc = spill_offsets(e, hl, offs, &stotal);
    (void)hipFree(hl); (void)hipFree(offs);
    if (rc) return rc;
    *bytes = ckpt_bytes(e->n, total, stotal);
    return 0;
}

extern "C" int gc_env_save(gc_env* e, void* buf, uint64_t cap, uint64_t* written) {
    if (!e || !buf) return fail("null argument");
    SRV_QUIESCE(e);
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    const int n = e->n;
    uint32_t *hl = nullptr, *offs = nullptr, *bad = nullptr, *scnt = nullptr, *soffs = nullptr, *fill = nullptr;
    u64 *ents = nullptr, *sents = nullptr;
    auto release = [&]() {
        (void)hipFree(hl); (void)hipFree(offs); (void)hipFree(bad); (void)hipFree(ents);
        (void)hipFree(scnt); (void)hipFree(soffs); (void)hipFree(fill); (void)hipFree(sents);
    };
    if (dalloc(&hl, n) || dalloc(&offs, n) || dalloc(&bad, 1) || dalloc(&scnt, n) || dalloc(&soffs, n) ||
        dalloc(&fill, n)) { release(); return -1; }
    uint64_t total = 0, stotal = 0;
    if (ckpt_offsets(e, e->meta, hl, offs, &total) || spill_offsets(e, scnt, soffs, &stotal)) { release(); return -1; }
    const size_t need = ckpt_bytes(n, total, stotal);
    if (written) *written = need;
    if (cap < need) { release(); return fail("checkpoint buffer too small: need " + std::to_string(need) + " bytes"); }
    if (dalloc(&ents, 8 * (total ? total : 1)) || dalloc(&sents, 8 * (stotal ? stotal : 1))) { release(); return -1; }
    CkptHeader hd = {};
    memcpy(hd.magic, CKPT_MAGIC, 8);
    hd.version = 2; hd.n = (uint32_t)n; hd.rules = (uint32_t)e->rules; hd.opp = (uint32_t)e->d.opp;
    hd.agent_black = (uint32_t)e->d.agent_black; hd.policy_ready = e->policy_ready ? 1u : 0u;
    hd.seed = e->seed;
    for (int j = 0; j < NBB; j++) hd.init[j] = e->d.init[j];
    hd.entries = total;
    hd.spill_entries = stotal;
    hd.layout = CKPT_LAYOUT;
    uint8_t* out = static_cast<uint8_t*>(buf);
    memcpy(out, &hd, sizeof hd);
    const size_t o_slab = sizeof hd, o_scnt = o_slab + Slab::BYTES_PER_BOARD * (size_t)n, o_ent = o_scnt + 4 * (size_t)n,
                 o_sent = o_ent + 64 * (size_t)total;
    uint32_t flag = 0;
    hipError_t he = hipMemsetAsync(bad, 0, 4, e->stream);
    if (he == hipSuccess) {
        k_ckpt_pack<<<grid_for(n), BLOCK, 0, e->stream>>>(e->d.htab, e->d.hgen, e->meta, n, e->d.hbits, offs, ents, bad);
        he = hipGetLastError();
    }
    if (he == hipSuccess && stotal) {
        const SpillTab& sp = e->d.ic.spill;
        const size_t slots = (size_t)sp.mask + 1;
        he = hipMemsetAsync(fill, 0, (size_t)4 * n, e->stream);
        if (he == hipSuccess) {
            k_spill_collect<<<(unsigned)((slots + BLOCK - 1) / BLOCK), BLOCK, 0, e->stream>>>(sp.ent, sp.mask, e->d.hgen,
                                                                                              fill, soffs, sents);
            he = hipGetLastError();
        }
    }
    if (he == hipSuccess) he = hipMemcpyAsync(out + o_slab, e->slab, Slab::BYTES_PER_BOARD * (size_t)n, hipMemcpyDeviceToHost, e->stream);
    if (he == hipSuccess) he = hipMemcpyAsync(out + o_scnt, scnt, 4 * (size_t)n, hipMemcpyDeviceToHost, e->stream);
    if (he == hipSuccess && total) he = hipMemcpyAsync(out + o_ent, ents, 64 * total, hipMemcpyDeviceToHost, e->stream);
    if (he == hipSuccess && stotal) he = hipMemcpyAsync(out + o_sent, sents, 64 * stotal, hipMemcpyDeviceToHost, e->stream);
    if (he == hipSuccess) he = hipMemcpyAsync(&flag, bad, 4, hipMemcpyDeviceToHost, e->stream);
    if (he == hipSuccess) he = hipStreamSynchronize(e->stream);
    release();
    if (he != hipSuccess) return fail(std::string("checkpoint save: ") + hipGetErrorString(he));
    if (flag) return fail("checkpoint save: a repetition window does not match its recorded length");
    return 0;
}

extern "C" int gc_env_load(gc_env* e, const void* buf, uint64_t size) {
    if (!e || !buf) return fail("null argument");
    SRV_QUIESCE(e);
    if (size < sizeof(CkptHeader)) return fail("checkpoint: truncated header");
    CkptHeader hd;
    memcpy(&hd, buf, sizeof hd);
    if (memcmp(hd.magic, CKPT_MAGIC, 8) != 0 || hd.version != 2) return fail("checkpoint: not a gc_env checkpoint (v2)");
    if (hd.layout != CKPT_LAYOUT) return fail("checkpoint: written by a build with another slab layout");
    if ((int)hd.n != e->n) return fail("checkpoint: it holds " + std::to_string(hd.n) + " boards, the env " + std::to_string(e->n));
    if ((int)hd.rules != e->rules || (int)hd.opp != e->d.opp || (int)hd.agent_black != e->d.agent_black)
        return fail("checkpoint: rules / opponent / player colour differ from the env's");
    if (hd.seed != e->seed) return fail("checkpoint: the env's seed differs (the policy streams would not continue)");
    for (int j = 0; j < NBB; j++)
        if (hd.init[j] != e->d.init[j]) return fail("checkpoint: the env's initial board differs");
    if (size != ckpt_bytes(e->n, hd.entries, hd.spill_entries)) return fail("checkpoint: size does not match its header");
    if (hd.spill_entries && !e->d.ic.spill.ent) return fail("checkpoint: spill entries, but the env has no spill table");
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    const int n = e->n;
    const uint8_t* in = static_cast<const uint8_t*>(buf);
    const size_t o_slab = sizeof hd, o_scnt = o_slab + Slab::BYTES_PER_BOARD * (size_t)n, o_ent = o_scnt + 4 * (size_t)n,
                 o_sent = o_ent + 64 * (size_t)hd.entries;
    uint8_t* slab = nullptr;
    u64 *ents = nullptr, *sents = nullptr;
    uint32_t *hl = nullptr, *offs = nullptr, *gnew = nullptr, *bad = nullptr, *scnt = nullptr, *soffs = nullptr;
    auto release = [&]() {
        (void)hipFree(slab); (void)hipFree(ents); (void)hipFree(hl); (void)hipFree(offs); (void)hipFree(gnew);
        (void)hipFree(bad); (void)hipFree(sents); (void)hipFree(scnt); (void)hipFree(soffs);
    };
    if (dalloc(&slab, Slab::BYTES_PER_BOARD * (size_t)n) || dalloc(&ents, 8 * (hd.entries ? hd.entries : 1)) ||
        dalloc(&sents, 8 * (hd.spill_entries ? hd.spill_entries : 1)) || dalloc(&hl, n) || dalloc(&offs, n) ||
        dalloc(&gnew, n) || dalloc(&bad, 1) || dalloc(&scnt, n) || dalloc(&soffs, n)) {
        release();
        return -1;
    }
    // stage everything and validate it against the env's tables before touching the env
    hipError_t he = hipMemcpyAsync(slab, in + o_slab, Slab::BYTES_PER_BOARD * (size_t)n, hipMemcpyHostToDevice, e->stream);
    if (he == hipSuccess) he = hipMemcpyAsync(scnt, in + o_scnt, 4 * (size_t)n, hipMemcpyHostToDevice, e->stream);
    if (he == hipSuccess && hd.entries)
        he = hipMemcpyAsync(ents, in + o_ent, 64 * hd.entries, hipMemcpyHostToDevice, e->stream);
    if (he == hipSuccess && hd.spill_entries)
        he = hipMemcpyAsync(sents, in + o_sent, 64 * hd.spill_entries, hipMemcpyHostToDevice, e->stream);
    if (he != hipSuccess) { release(); return fail(std::string("checkpoint load: ") + hipGetErrorString(he)); }
    uint64_t total = 0, stotal = 0;
    const u32* smeta = reinterpret_cast<const u32*>(slab + Slab::meta(n));
    if (ckpt_offsets(e, smeta, hl, offs, &total) || scan_u32(e, scnt, soffs, n, &stotal)) { release(); return -1; }
    if (total != hd.entries || stotal != hd.spill_entries) {
        release();
        return fail("checkpoint: window lengths do not match the entries it holds");
    }
    uint32_t flag = 0;
    he = hipMemsetAsync(bad, 0, 4, e->stream);
    if (he == hipSuccess) {
        k_ckpt_check<<<grid_for(n), BLOCK, 0, e->stream>>>(smeta, scnt, n, e->d.hbits, e->d.ic.spill.ent != nullptr, bad);
        he = hipGetLastError();
    }
    if (he == hipSuccess) he = hipMemcpyAsync(&flag, bad, 4, hipMemcpyDeviceToHost, e->stream);
    if (he == hipSuccess) he = hipStreamSynchronize(e->stream);
    if (he != hipSuccess || flag) {
        release();
        return fail(he != hipSuccess ? std::string("checkpoint load: ") + hipGetErrorString(he)
                                     : std::string("checkpoint: its repetition windows do not fit this env's tables"));
    }
    // the spill table, emptied (every entry would be dead under the fresh generations) and
    // sized for the restored entries at a load <= 1/8
    if (e->d.ic.spill.ent) {
        int bits = e->sp_bits;
        while (((uint64_t)1 << bits) < 8 * stotal) bits++;
        if (spill_alloc(e, bits)) { release(); return -1; }
    }
    // from here on the env changes; a failure resets every board (never a half-restored env)
    k_ckpt_gen<<<grid_for(n), BLOCK, 0, e->stream>>>(e->d.hgen, reinterpret_cast<const u32*>(slab + Slab::hgen(n)), n,
                                                     gnew);
    he = hipGetLastError();
    if (he == hipSuccess)
        he = hipMemcpyAsync(e->slab, slab, Slab::BYTES_PER_BOARD * (size_t)n, hipMemcpyDeviceToDevice, e->stream);
    if (he == hipSuccess) he = hipMemsetAsync(bad, 0, 4, e->stream);
    if (he == hipSuccess) {
        k_ckpt_unpack<<<grid_for(n), BLOCK, 0, e->stream>>>(e->d.htab, e->d.hgen, e->meta, n, e->d.hbits, gnew, offs,
                                                            ents, e->d.ic.spill, stotal ? scnt : nullptr, soffs, sents,
                                                            bad);
        he = hipGetLastError();
    }
    if (he == hipSuccess) he = hipMemcpyAsync(&flag, bad, 4, hipMemcpyDeviceToHost, e->stream);
    if (he == hipSuccess) he = hipStreamSynchronize(e->stream);
    release();
    if (he != hipSuccess || flag) {
        std::string m = he != hipSuccess ? std::string("checkpoint load: ") + hipGetErrorString(he)
                                         : std::string("checkpoint load: a repetition window did not fit the table");
        if (he == hipSuccess) {  // the env is half-restored: start every board afresh
            launch_reset(e, nullptr, 1);
            (void)hipStreamSynchronize(e->stream);
            e->policy_ready = true;
            m += " (every board was reset)";
        }
        return fail(m);
    }
    e->policy_ready = hd.policy_ready != 0;
    return 0;
}

// bytes of device memory held by the env (for reports)
extern "C" uint64_t gc_env_device_bytes(gc_env* e) {
    if (!e) return 0;
    uint64_t n = (uint64_t)e->n;
    return n * (NBB * 8 + 4) + n * ((uint64_t)64 << e->d.hbits) + n * (4 + 4 + 2 + 4 + 1 + 1 + 4) +
           n * (64 + 8 + 1 + 4 + 64);
}
