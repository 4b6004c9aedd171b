// Diagnostic only: static instruction cost of each gc_core function, one per tiny kernel
// (compile with -S and count: tools/cost_model.sh).  Loops count once (per-iteration cost).
#include <hip/hip_runtime.h>

#include "../gym-chess_amd/csrc/gc_core.h"
#include "../gym-chess_amd/csrc/gc_env.h"
using namespace gc;

struct S {
    static constexpr bool kPark = true;
    u64* base;
    __device__ void put(int j, u64 v) { base[j * 64] = v; }
    __device__ u64 get(int j) const { return base[j * 64]; }
};
__device__ Pos ld(const u64* p) {
    int i = threadIdx.x;
    Pos s;
    s.k = p[i]; s.q = p[i + 64]; s.r = p[i + 128]; s.b = p[i + 192]; s.n = p[i + 256]; s.p = p[i + 320];
    s.w = p[i + 384]; s.meta = (u32)p[i + 448];
    return s;
}
extern "C" __global__ void c_side_attacks(const u64* p, u64* o) { Pos s = ld(p); o[threadIdx.x] = side_attacks(s, s.meta & 1); }
extern "C" __global__ void c_gen_base(const u64* p, u64* o) {
    Pos s = ld(p); Gen g; gen_base(s, g); o[threadIdx.x] = g.own ^ g.opp ^ (u64)g.ks;
}
extern "C" __global__ void c_gen_pins(const u64* p, u64* o) {
    Pos s = ld(p); Gen g; gen_base(s, g); gen_pins(s, g); o[threadIdx.x] = g.checkmask ^ g.pinned ^ g.pinrays;
}
extern "C" __global__ void c_gen_enemy(const u64* p, u64* o) {
    Pos s = ld(p); Gen g; gen_base(s, g); gen_enemy(s, g); o[threadIdx.x] = g.enemy_att ^ g.castles;
}
extern "C" __global__ void c_sq_attacked(const u64* p, u64* o) { Pos s = ld(p); o[threadIdx.x] = sq_attacked(s, (int)(s.meta & 63), true); }
extern "C" __global__ void c_apply_legal(const u64* p, u64* o) {
    Pos s = ld(p); int r; bool ir; apply_legal(s, true, (int)(p[512 + threadIdx.x] & 4095), &r, &ir);
    o[threadIdx.x] = s.k ^ s.q ^ s.r ^ s.b ^ s.n ^ s.p ^ s.w ^ s.meta ^ (u64)r ^ (u64)ir;
}
extern "C" __global__ void c_board_key(const u64* p, u64* o) { Pos s = ld(p); o[threadIdx.x] = board_key(s); }
extern "C" __global__ void c_philox(const u64* p, u64* o) { o[threadIdx.x] = philox_x0(p[0], threadIdx.x, (u32)p[1]); }
extern "C" __global__ void c_gen_moves_a(const u64* p, u64* o) {
    __shared__ u64 L[16 * 64];
    S sc{L + threadIdx.x}; Pos s = ld(p); Gen g; gen_init(s, g); MoveSet ms; moveset_clear(ms);
    o[threadIdx.x] = gen_moves_a(s, g, ms, sc) ^ ms.cnt[0] ^ ms.cnt[1] ^ ms.cnt[2] ^ ms.cnt[3] ^ ms.cnt[4] ^ ms.o1 ^ ms.o2 ^
                     ms.ol ^ ms.orr;
}
extern "C" __global__ void c_gen_moves_b(const u64* p, u64* o) {
    __shared__ u64 L[16 * 64];
    S sc{L + threadIdx.x}; Pos s = ld(p); Gen g; gen_init(s, g); MoveSet ms; moveset_clear(ms);
    o[threadIdx.x] = gen_moves_b(s, g, ms, sc) ^ ms.cnt[0] ^ ms.cnt[1] ^ ms.cnt[2] ^ ms.cnt[3] ^ ms.cnt[4];
}
extern "C" __global__ void c_select_action(const u64* p, u64* o) {
    __shared__ u64 L[16 * 64];
    S sc{L + threadIdx.x}; Pos s = ld(p); Gen g; g.white = 1; g.own = p[600]; g.castles = 3; MoveSet ms;
    ms.fastp = p[601]; ms.o1 = p[602]; ms.o2 = p[603]; ms.ol = p[604]; ms.orr = p[605];
    for (int b = 0; b < 5; b++) ms.cnt[b] = p[606 + b];
    ms.total = (int)p[611]; ms.big = false;
    o[threadIdx.x] = select_action(s, g, ms, sc, (int)(p[612 + threadIdx.x] & 31));
}
// perft leaf pieces: the count of a position given its context, the child's context, a child
extern "C" __global__ void c_count_moves(const u64* p, u64* o) {
    Pos s = ld(p); Gen g; gen_init(s, g); o[threadIdx.x] = (u64)count_moves(s, g);
}
extern "C" __global__ void c_gen_init(const u64* p, u64* o) {
    Pos s = ld(p); Gen g; gen_init(s, g);
    o[threadIdx.x] = g.checkmask ^ g.pinned ^ g.pinrays ^ g.enemy_att ^ g.castles ^ (u64)g.ks;
}
extern "C" __global__ void c_child_count(const u64* p, u64* o) {
    Pos s = ld(p); int r; bool ir;
    apply_legal(s, true, (int)(p[512 + threadIdx.x] & 4095), &r, &ir);
    s.meta = (s.meta & ~(u32)M_RIGHTS) | eff_rights(s);
    Gen g; gen_init(s, g); o[threadIdx.x] = (u64)count_moves(s, g);
}
extern "C" __global__ void c_count_position(const u64* p, u64* o) { Pos s = ld(p); o[threadIdx.x] = (u64)count_position(s); }
