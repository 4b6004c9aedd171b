/*
 * gc_oracle.c -- TEST INFRASTRUCTURE ONLY (parity oracle + CPU baseline).
 *
 * A plain-C, scalar, mailbox restatement of the reference chess engine
 * (/root/reference/src/lib.rs, the PyO3 `gym_chess.gym_chess` module) and of the
 * env bookkeeping of /root/reference/gym_chess/envs/chess_v2.py.  It keeps the
 * reference's *procedure* (per-square probes, per-move legality filter by
 * next_state + full attack-map recompute, row-major scan order) so that move
 * ORDER, next states, rewards and perft counts are reproduced bit-exactly,
 * including every rule quirk listed in SURVEY.md §0 (Q1-Q10).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library.  The product path (gym-chess_amd/) never links or calls it.
 *
 * Pinned by: tests/golden/ JSON fixtures (generated from the importable v1 reference,
 * the reference's own v2 known-answer tests, and the v2 env driven over this
 * engine) -- see tests/golden/make_golden.py and DESIGN.md "Oracle".
 *
 * Square numbering: sq = row*8 + col, row 0 = rank 8 (lib.rs:1235-1238).
 * Actions: from*64+to; 4096 KSW, 4097 QSW, 4098 KSB, 4099 QSB (chess_v2.py:492-506).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <stdatomic.h>

#define EMPTY 0
#define KING 1
#define QUEEN 2
#define ROOK 3
#define BISHOP 4
#define KNIGHT 5
#define PAWN 6

#define WHITE 1
#define BLACK (-1)

#define A_KSW 4096
#define A_QSW 4097
#define A_KSB 4098
#define A_QSB 4099

#define MAXMOVES 1024

/* lib.rs:281-293 */
typedef struct {
    int8_t b[64];
    int8_t player;           /* +1 white, -1 black */
    uint8_t wk_on, bk_on;    /* white/black king on board */
    uint8_t wkc, wqc, bkc, bqc;
    uint8_t wchk, bchk;
} OState;

typedef struct { uint8_t f, t; } OMove;

/* lib.rs:19-25 values, indexed by |id| */
static const int VALUE[7] = {0, 0, 10, 5, 3, 3, 1};

static int color_of(int id) { return id > 0 ? WHITE : (id < 0 ? BLACK : 0); }
static int type_of(int id) { return id < 0 ? -id : id; }
static int on_board(int r, int c) { return !(r < 0 || r > 7 || c < 0 || c > 7); } /* lib.rs:1190 */

/* lib.rs:1201-1210 is_piece_from_player (kings included: Q7) */
static int is_piece_from_player(const OState *s, int player, int r, int c) {
    int id = s->b[r * 8 + c];
    if (id == 0) return 0;
    return color_of(id) == player;
}
/* lib.rs:1217-1228 */
static int is_king_from_player(const OState *s, int player, int r, int c) {
    int id = s->b[r * 8 + c];
    if (type_of(id) != KING || id == 0) return 0;
    return color_of(id) == player;
}

static int piece_is_on_board(const int8_t *b, int id) { /* lib.rs:1375-1384 */
    for (int i = 0; i < 64; i++) if (b[i] == id) return 1;
    return 0;
}

/* State::new, lib.rs:295-336: king-on-board recomputed, rights forced false w/o king */
void o_state_new(OState *s, const int8_t *board, int player, int wkc, int wqc, int bkc, int bqc) {
    memcpy(s->b, board, 64);
    s->player = (int8_t)player;
    s->wk_on = (uint8_t)piece_is_on_board(board, KING);
    s->bk_on = (uint8_t)piece_is_on_board(board, -KING);
    s->wkc = (uint8_t)(wkc && s->wk_on);
    s->wqc = (uint8_t)(wqc && s->wk_on);
    s->bkc = (uint8_t)(bkc && s->bk_on);
    s->bqc = (uint8_t)(bqc && s->bk_on);
    s->wchk = 0;
    s->bchk = 0;
}

/* ---- probes ---------------------------------------------------------- */
/* lib.rs:1063-1081 playable_move -> add, stop */
static void playable_move(const OState *s, int player, int r, int c, int *add, int *stop) {
    if (!on_board(r, c)) { *add = 0; *stop = 1; return; }
    if (s->b[r * 8 + c] == 0) { *add = 1; *stop = 0; return; }
    if (is_piece_from_player(s, player, r, c)) { *add = 0; *stop = 1; return; }
    /* other player's piece, kings included (Q7) */
    *add = 1; *stop = 1;
}
/* lib.rs:1089-1104 attacking_move: every piece stops a ray and is included */
static void attacking_move(const OState *s, int player, int r, int c, int *add, int *stop) {
    (void)player;
    if (!on_board(r, c)) { *add = 0; *stop = 1; return; }
    if (s->b[r * 8 + c] == 0) { *add = 1; *stop = 0; return; }
    *add = 1; *stop = 1;
}
/* lib.rs:1113-1140 king_playable_move */
static int king_playable_move(const OState *s, int player, int r, int c, const uint8_t *amap) {
    if (!on_board(r, c)) return 0;
    if (amap[r * 8 + c]) return 0;
    if (s->b[r * 8 + c] == 0 || is_piece_from_player(s, -player, r, c)) return 1;
    return 0; /* own piece */
}
/* lib.rs:1147-1174 king_attacking_move: amap is always empty in attack mode */
static int king_attacking_move(const OState *s, int player, int r, int c, const uint8_t *amap) {
    (void)s; (void)player;
    if (!on_board(r, c)) return 0;
    if (amap && amap[r * 8 + c]) return 0;
    return 1;
}

/* ---- per-piece generators (append in reference order) --------------- */
typedef struct { OMove m[MAXMOVES]; int n; } OList;

static void push(OList *L, int fr, int fc, int tr, int tc) {
    if (L->n < MAXMOVES) { L->m[L->n].f = (uint8_t)(fr * 8 + fc); L->m[L->n].t = (uint8_t)(tr * 8 + tc); L->n++; }
}

static const int KING_STEPS[8][2] = {{1,0},{-1,0},{0,1},{0,-1},{1,1},{1,-1},{-1,1},{-1,-1}}; /* lib.rs:797-806 */
static const int ROOK_STEPS[4][2] = {{-1,0},{1,0},{0,-1},{0,1}};                              /* lib.rs:835 */
static const int BISHOP_STEPS[4][2] = {{-1,-1},{-1,1},{1,-1},{1,1}};                          /* lib.rs:845 */
static const int KNIGHT_STEPS[8][2] = {{-2,-1},{-2,1},{2,-1},{2,1},{-1,-2},{-1,2},{1,-2},{1,2}}; /* lib.rs:891-900 */

static void king_moves(const OState *s, int player, int r, int c, const uint8_t *amap, int attack, OList *L) {
    for (int k = 0; k < 8; k++) {
        int tr = r + KING_STEPS[k][0], tc = c + KING_STEPS[k][1];
        int add = attack ? king_attacking_move(s, player, tr, tc, amap) : king_playable_move(s, player, tr, tc, amap);
        if (add) push(L, r, c, tr, tc);
    }
}
static void iterativesteps(const OState *s, int player, int r, int c, int dr, int dc, int attack, OList *L) {
    for (int k = 1;; k++) { /* lib.rs:853-887 */
        int tr = r + k * dr, tc = c + k * dc, add, stop;
        if (attack) attacking_move(s, player, tr, tc, &add, &stop);
        else playable_move(s, player, tr, tc, &add, &stop);
        if (add) push(L, r, c, tr, tc);
        if (stop) break;
    }
}
static void rook_moves(const OState *s, int player, int r, int c, int attack, OList *L) {
    for (int k = 0; k < 4; k++) iterativesteps(s, player, r, c, ROOK_STEPS[k][0], ROOK_STEPS[k][1], attack, L);
}
static void bishop_moves(const OState *s, int player, int r, int c, int attack, OList *L) {
    for (int k = 0; k < 4; k++) iterativesteps(s, player, r, c, BISHOP_STEPS[k][0], BISHOP_STEPS[k][1], attack, L);
}
static void knight_moves(const OState *s, int player, int r, int c, int attack, OList *L) {
    for (int k = 0; k < 8; k++) { /* lib.rs:889-916 */
        int tr = r + KNIGHT_STEPS[k][0], tc = c + KNIGHT_STEPS[k][1], add, stop;
        if (attack) attacking_move(s, player, tr, tc, &add, &stop);
        else playable_move(s, player, tr, tc, &add, &stop);
        if (add) push(L, r, c, tr, tc);
    }
}
/* lib.rs:918-964 (Q1: double push checks only the destination; Q3 no e.p.) */
static void pawn_moves(const OState *s, int player, int r, int c, int attack, OList *L) {
    int p = player;
    int ar[2] = {r - p, r - p}, ac[2] = {c + 1, c - 1};
    if (attack) {
        for (int k = 0; k < 2; k++)
            if (on_board(ar[k], ac[k]) && !is_king_from_player(s, player, ar[k], ac[k])) push(L, r, c, ar[k], ac[k]);
        return;
    }
    int or_ = r - p, tr2 = r - 2 * p;
    if (on_board(or_, c) && s->b[or_ * 8 + c] == 0) push(L, r, c, or_, c);
    if (on_board(tr2, c) && ((player == WHITE && r == 6) || (player == BLACK && r == 1)) && s->b[tr2 * 8 + c] == 0)
        push(L, r, c, tr2, c);
    for (int k = 0; k < 2; k++)
        if (on_board(ar[k], ac[k]) && is_piece_from_player(s, -player, ar[k], ac[k])) push(L, r, c, ar[k], ac[k]);
}

/* lib.rs:501-555 (scan + dispatch; the filter is applied by the caller) */
static void raw_moves(const OState *s, int player, int attack, const uint8_t *amap, OList *L) {
    L->n = 0;
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++) {
            int id = s->b[i * 8 + j];
            if (id == 0 || color_of(id) != player) continue;
            switch (type_of(id)) {
            case KING: king_moves(s, player, i, j, amap, attack, L); break;
            case QUEEN: rook_moves(s, player, i, j, attack, L); bishop_moves(s, player, i, j, attack, L); break;
            case ROOK: rook_moves(s, player, i, j, attack, L); break;
            case BISHOP: bishop_moves(s, player, i, j, attack, L); break;
            case KNIGHT: knight_moves(s, player, i, j, attack, L); break;
            case PAWN: pawn_moves(s, player, i, j, attack, L); break;
            }
        }
}

/* lib.rs:669-677 get_squares_under_attack_by_player */
void o_attack_map(const OState *s, int player, uint8_t *amap) {
    static const uint8_t EMPTY_MAP[64] = {0};
    OList L;
    raw_moves(s, player, 1, EMPTY_MAP, &L);
    memset(amap, 0, 64);
    for (int k = 0; k < L.n; k++) amap[L.m[k].t] = 1;
}

/* lib.rs:634-667 _king_is_checked. NB the `break` leaves only the inner loop,
 * so with several kings the LAST row holding one wins (first such square in it). */
static int king_is_checked_map(const OState *s, int player, const uint8_t *amap) {
    int ks = -1, kid = KING * player;
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++)
            if (s->b[i * 8 + j] == kid) { ks = i * 8 + j; break; }
    if (ks < 0) return 0;
    return amap[ks] != 0;
}
/* lib.rs:628-632 */
static int king_is_checked(const OState *s, int player) {
    uint8_t amap[64];
    o_attack_map(s, -player, amap);
    return king_is_checked_map(s, player, amap);
}

/* lib.rs:679-784 next_state (no legality check; `player` is the caller's, not the piece's).
 * castle: 0 = normal, else action code 4096..4099. Returns 0 ok, -1 empty from-square (panic). */
int o_next_state(const OState *in, int player, int action, OState *out, int *reward) {
    *out = *in;
    *reward = 0;
    if (action < 4096) {
        int f = action / 64, t = action % 64;
        int piece = out->b[f];
        int cap = out->b[t];
        if (piece == 0) return -1; /* lib.rs:693-695 panic */
        out->b[f] = 0;
        out->b[t] = (int8_t)piece;
        *reward += VALUE[type_of(cap)];
        /* lib.rs:700-709 promotion (inverted rows: dead in generated play, Q2) */
        if (type_of(piece) == PAWN) {
            if ((player == WHITE && t / 8 == 7) || (player == BLACK && t / 8 == 0)) {
                out->b[t] = (int8_t)(QUEEN * player);
                *reward += 10;
            }
        }
        /* lib.rs:711-734 rights: only POSITIVE ids compared (Q5) */
        if (piece == KING) {
            if (player == WHITE) { out->wkc = 0; out->wqc = 0; }
            else { out->bkc = 0; out->bqc = 0; }
        } else if (piece == ROOK) {
            if (f % 8 == 0) { if (player == WHITE) out->wqc = 0; else out->bqc = 0; }
            else if (f % 8 == 7) { if (player == WHITE) out->wkc = 0; else out->bkc = 0; }
        }
    } else {
        int8_t *b = out->b;
        switch (action) { /* lib.rs:740-773 */
        case A_KSW: b[60] = 0; b[61] = ROOK; b[62] = KING; b[63] = 0; out->wkc = out->wqc = 0; break;
        case A_QSW: b[56] = 0; b[57] = 0; b[58] = KING; b[59] = ROOK; b[60] = 0; out->wkc = out->wqc = 0; break;
        case A_KSB: b[4] = 0; b[5] = -ROOK; b[6] = -KING; b[7] = 0; out->bkc = out->bqc = 0; break;
        case A_QSB: b[0] = 0; b[1] = 0; b[2] = -KING; b[3] = -ROOK; b[4] = 0; out->bkc = out->bqc = 0; break;
        default: return -2;
        }
    }
    out->player = (int8_t)(-player); /* lib.rs:778-780 */
    return 0;
}

/* lib.rs:612-626 */
static int move_leaves_king_checked(const OState *s, int player, OMove m) {
    if ((player == WHITE && s->b[m.f] == KING) || (player == BLACK && s->b[m.f] == -KING)) return 0;
    OState ns;
    int rw;
    o_next_state(s, player, m.f * 64 + m.t, &ns, &rw);
    return king_is_checked(&ns, player);
}

/* lib.rs:966-1056 calc_castle_moves (Q4: black tests the POSITIVE ids) */
static int calc_castle_moves(const OState *s, int player, const uint8_t *amap, uint16_t *out) {
    int n = 0;
    const int8_t *b = s->b;
    if (player == WHITE) {
        if (b[56] == ROOK && b[57] == 0 && b[58] == 0 && b[59] == 0 && b[60] == KING && !amap[60] && !amap[59] && !amap[58])
            out[n++] = A_QSW;
        if (b[63] == ROOK && b[62] == 0 && b[61] == 0 && b[60] == KING && !amap[60] && !amap[61] && !amap[62])
            out[n++] = A_KSW;
    } else {
        if (b[0] == ROOK && b[1] == 0 && b[2] == 0 && b[3] == 0 && b[4] == KING && !amap[4] && !amap[3] && !amap[2])
            out[n++] = A_QSB;
        if (b[7] == ROOK && b[6] == 0 && b[5] == 0 && b[4] == KING && !amap[4] && !amap[5] && !amap[6])
            out[n++] = A_KSB;
    }
    return n;
}

/* lib.rs:578-610 _get_possible_castle_moves (Q5: OR of the two rights) */
static int castle_moves(const OState *s, int player, int attack, const uint8_t *amap, uint16_t *out) {
    if (attack) return 0;
    if ((player == WHITE && !s->wk_on) || (player == BLACK && !s->bk_on)) return 0;
    if ((player == WHITE && (s->wkc || s->wqc)) || (player == BLACK && (s->bkc || s->bqc)))
        return calc_castle_moves(s, player, amap, out);
    return 0;
}

/* lib.rs:460-486 + 1454-1480: ordered action list (normal moves, then castles). */
int o_get_possible_moves(const OState *s, int player, int attack, uint16_t *out, int cap) {
    static const uint8_t EMPTY_MAP[64] = {0};
    uint8_t amap[64];
    const uint8_t *m = EMPTY_MAP;
    if (!attack) { o_attack_map(s, -player, amap); m = amap; }
    OList Ls, *L = &Ls;
    raw_moves(s, player, attack, m, L);
    int n = 0;
    for (int k = 0; k < L->n; k++) {
        if (!attack && move_leaves_king_checked(s, player, L->m[k])) continue; /* lib.rs:561 */
        if (n < cap) out[n] = (uint16_t)(L->m[k].f * 64 + L->m[k].t);
        n++;
    }
    uint16_t cm[2];
    int nc = castle_moves(s, player, attack, m, cm);
    for (int k = 0; k < nc; k++) { if (n < cap) out[n] = cm[k]; n++; }
    return n;
}

int o_get_castle_moves(const OState *s, int player, uint16_t *out) { /* lib.rs:566-575 */
    uint8_t amap[64];
    o_attack_map(s, -player, amap);
    return castle_moves(s, player, 0, amap, out);
}

/* lib.rs:1386-1393 */
void o_update_state(OState *s) {
    uint8_t amap[64];
    o_attack_map(s, BLACK, amap);
    s->wchk = (uint8_t)king_is_checked_map(s, WHITE, amap);
    o_attack_map(s, WHITE, amap);
    s->bchk = (uint8_t)king_is_checked_map(s, BLACK, amap);
}

/* ====================================================================== */
/* Flat C ABI used by tests (oracle/oracle.py).  State in/out as            */
/* int8 board[64] + uint8 meta[8] = {player(1=W,0=B), wkc,wqc,bkc,bqc, wchk, bchk, 0} */
/* ====================================================================== */
static void meta_to_state(OState *s, const int8_t *board, const uint8_t *meta) {
    o_state_new(s, board, meta[0] ? WHITE : BLACK, meta[1], meta[2], meta[3], meta[4]);
}
static void state_to_meta(const OState *s, int8_t *board, uint8_t *meta) {
    memcpy(board, s->b, 64);
    meta[0] = s->player == WHITE;
    meta[1] = s->wkc; meta[2] = s->wqc; meta[3] = s->bkc; meta[4] = s->bqc;
    meta[5] = s->wchk; meta[6] = s->bchk; meta[7] = 0;
}

/* ChessEngine.get_possible_moves(state, player, attack) lib.rs:1454 */
int oracle_get_possible_moves(const int8_t *board, const uint8_t *meta, int player_white, int attack, uint16_t *out, int cap) {
    OState s;
    meta_to_state(&s, board, meta);
    return o_get_possible_moves(&s, player_white ? WHITE : BLACK, attack, out, cap);
}
/* ChessEngine.get_castle_moves lib.rs:1482 */
int oracle_get_castle_moves(const int8_t *board, const uint8_t *meta, int player_white, uint16_t *out) {
    OState s;
    meta_to_state(&s, board, meta);
    return o_get_castle_moves(&s, player_white ? WHITE : BLACK, out);
}
/* ChessEngine.next_state lib.rs:1422-1452. Returns 0 ok, 1 both-kings-checked (exception set),
 * -1 empty from-square (panic). */
int oracle_next_state(const int8_t *board, const uint8_t *meta, int player_white, int action,
                      int8_t *out_board, uint8_t *out_meta, int *reward) {
    OState s, ns;
    meta_to_state(&s, board, meta);
    int rc = o_next_state(&s, player_white ? WHITE : BLACK, action, &ns, reward);
    if (rc) return rc;
    o_update_state(&ns);
    state_to_meta(&ns, out_board, out_meta);
    return (ns.wchk && ns.bchk) ? 1 : 0;
}
/* ChessEngine.update_state lib.rs:1502-1511 */
void oracle_update_state(const int8_t *board, const uint8_t *meta, int8_t *out_board, uint8_t *out_meta) {
    OState s;
    meta_to_state(&s, board, meta);
    o_update_state(&s);
    state_to_meta(&s, out_board, out_meta);
}

/* perft by composition: moves from get_all_possible_moves, recurse on next_state */
static uint64_t perft_rec(const OState *s, int depth) {
    uint16_t mv[MAXMOVES];
    int n = o_get_possible_moves(s, s->player, 0, mv, MAXMOVES);
    if (depth <= 1) return (uint64_t)n;
    uint64_t tot = 0;
    for (int k = 0; k < n; k++) {
        OState ns, ns2;
        int rw;
        o_next_state(s, s->player, mv[k], &ns, &rw);
        /* the engine re-reads the dict each call: State::new forces rights by king presence */
        o_state_new(&ns2, ns.b, ns.player, ns.wkc, ns.wqc, ns.bkc, ns.bqc);
        tot += perft_rec(&ns2, depth - 1);
    }
    return tot;
}
uint64_t oracle_perft(const int8_t *board, const uint8_t *meta, int depth) {
    OState s;
    meta_to_state(&s, board, meta);
    if (depth <= 0) return 1;
    return perft_rec(&s, depth);
}

/* ====================================================================== */
/* Env layer: chess_v2.py ChessEnvV2, opponent "none" or the on-device random opponent     */
/* ====================================================================== */
typedef struct {
    OState st;               /* board, rights, checks; st.player = current_player */
    int done;
    int move_count;
    int8_t init[64];
    /* saved_boards (chess_v2.py:192, 404-407): board-only key */
    int8_t (*saved)[64];
    int *cnt;
    int nsaved, capsaved;
    uint16_t moves[MAXMOVES];
    int nmoves;
    /* opponent (chess_v2.py:167-181): 0 none, 1 random = the Philox policy below, drawing
     * from the same per-board stream (seed, board, draw++) as the self-play driver */
    int opp, agent_black;
    int set_order;  /* the policy's order: 1 move-set order, 0 action-id order (the API step's pick) */
    uint64_t seed;
    uint32_t board, draw;
    /* distinct pre-move boards of reversible moves since the last pawn move / capture: the
     * device's window length (unbounded: a BLACK agent's move_count never advances,
     * 291-292, so its games have no move cap and saved_boards grows for the whole game --
     * the device spills such windows past its per-board table, gc_env.h) */
    int win;
} OEnv;

uint32_t oracle_policy_index(uint64_t seed, uint32_t board, uint32_t draw, uint32_t n);
static int kth_in_action_order(const uint16_t *moves, int n, int k);

static void env_clear_saved(OEnv *e) { e->nsaved = 0; e->win = 0; }

static int env_saved_inc(OEnv *e, const int8_t *b) {
    for (int i = 0; i < e->nsaved; i++)
        if (memcmp(e->saved[i], b, 64) == 0) return ++e->cnt[i];
    if (e->nsaved == e->capsaved) {
        e->capsaved = e->capsaved ? 2 * e->capsaved : 64;
        e->saved = realloc(e->saved, (size_t)e->capsaved * 64);
        e->cnt = realloc(e->cnt, (size_t)e->capsaved * sizeof(int));
    }
    memcpy(e->saved[e->nsaved], b, 64);
    e->cnt[e->nsaved] = 1;
    return e->cnt[e->nsaved++];
}

/* state as the engine sees it on each FFI call (convert_py_state -> State::new) */
static void env_engine_state(const OEnv *e, OState *s) {
    o_state_new(s, e->st.b, e->st.player, e->st.wkc, e->st.wqc, e->st.bkc, e->st.bqc);
}

static int kth_in_set_order(const int8_t *b, const uint16_t *moves, int n, int k);

/* the random policy's pick (self-play and the opponent): uniform rank over the legal list, the
 * k-th legal action in move-set order (set_order 0: action-id order, the API step's `pick`) */
static int env_policy_pick(OEnv *e) {
    uint32_t k = oracle_policy_index(e->seed, e->board, e->draw++, (uint32_t)e->nmoves);
    if (e->set_order) return kth_in_set_order(e->st.b, e->moves, e->nmoves, (int)k);
    return kth_in_action_order(e->moves, e->nmoves, (int)k);
}

/* player_move (chess_v2.py:393-412) + the state setter + switch_player + the next
 * get_possible_moves: returns 1 on the both-kings-checked error (env unchanged), else 0
 * with *mr = capture value and *rep = the 3-fold verdict on the PRE-move board. */
static int env_player_move(OEnv *e, int action, int *mr, int *rep) {
    OState s, ns;
    env_engine_state(e, &s);
    int me = e->st.player;
    int irrev = action < 4096 && (type_of(e->st.b[action >> 6]) == PAWN || e->st.b[action & 63] != 0);
    o_next_state(&s, me, action, &ns, mr);                                               /* 419 */
    o_update_state(&ns);
    if (ns.wchk && ns.bchk) return 1;                                                    /* lib.rs:1442 */
    int c = env_saved_inc(e, e->st.b);
    *rep = c >= 3;                                                                       /* 404-407 */
    if (irrev) e->win = 0;
    else if (c == 1) e->win++;
    /* state setter (315-323): board, rights, checks; current_player is NOT taken from the dict */
    memcpy(e->st.b, ns.b, 64);
    e->st.wkc = ns.wkc; e->st.wqc = ns.wqc; e->st.bkc = ns.bkc; e->st.bqc = ns.bqc;
    e->st.wchk = ns.wchk; e->st.bchk = ns.bchk;
    e->st.player = (int8_t)(-me);                                                        /* switch_player */
    OState s2;
    env_engine_state(e, &s2);
    e->nmoves = o_get_possible_moves(&s2, e->st.player, 0, e->moves, MAXMOVES);
    return 0;
}

/* chess_v2.py:183-217.  With player_color=BLACK the opponent opens as WHITE (208-216):
 * its move counts for 3-fold, its `done` is discarded, move_count becomes 1.  An opening
 * position without a legal move makes the reference's policy return "resign" and crash;
 * here that marks the env done (reason 9 is reported by the next step). */
void o_env_reset(OEnv *e) {
    OState s;
    o_state_new(&s, e->init, WHITE, 1, 1, 1, 1);
    o_update_state(&s); /* engine.update_state(self.state) */
    e->st = s;
    e->done = 0;
    e->move_count = 0;
    env_clear_saved(e);
    e->nmoves = o_get_possible_moves(&e->st, WHITE, 0, e->moves, MAXMOVES);
    if (e->opp && e->agent_black) {
        if (e->nmoves == 0) { e->done = 1; return; }
        int mr, rep;
        if (env_player_move(e, env_policy_pick(e), &mr, &rep) == 1) { e->done = 1; return; }
        e->move_count = 1;
    }
}

/* chess_v2.py:219-294.
 * Returns status: 0 ok, 1 both-kings-checked error (the reference raises SystemError).
 * reward / done out.  Reason: 0 none, 1 opponent mated (+100), 2 3-fold, 3 move cap,
 * 6 invalid action, 7 already done, 8 agent mated by the opponent's reply (-100),
 * 9 the opponent has no legal reply and no check (the reference's policy returns "resign",
 * which maps to no action: the reference raises; here the env ends). */
int o_env_step(OEnv *e, int action, int *reward, int *done, int *reason) {
    *reason = 0;
    int valid = 0;
    for (int k = 0; k < e->nmoves; k++) if (e->moves[k] == action) { valid = 1; break; }
    if (!valid) { *reward = -10; *done = e->done; *reason = 6; return 0; }           /* 240-242 */
    if (e->done) { *reward = 0; *done = 1; *reason = 7; return 0; }                  /* 245-251 */
    if (e->move_count > 149) { *reward = 0; *done = 1; *reason = 3; return 0; }       /* 252-258 */
    int rw = -10;                                                                       /* 261 (Q9) */
    int mr, rep;
    int pm = env_player_move(e, action, &mr, &rep);
    if (pm == 1) { *reward = 0; *done = 0; return 1; }
    e->done = rep;
    if (rep) *reason = 2;
    rw += mr;
    int opp_chk = e->st.player == WHITE ? e->st.wchk : e->st.bchk;
    if (e->nmoves == 0 && opp_chk) { e->done = 1; rw += 100; *reason = 1; }              /* 270-272 */
    if (e->done) { *reward = rw; *done = 1; return 0; }
    if (e->opp) {                                                                        /* 275-288 */
        if (e->nmoves == 0) { e->done = 1; *reward = rw; *done = 1; *reason = 9; return 0; }
        int omr, orep;
        pm = env_player_move(e, env_policy_pick(e), &omr, &orep);
        if (pm == 1) { *reward = rw; *done = 1; return 1; }
        e->done = orep;
        if (orep) *reason = 2;
        rw -= omr;
        int my_chk = e->st.player == WHITE ? e->st.wchk : e->st.bchk;
        if (e->nmoves == 0 && my_chk) { e->done = 1; rw -= 100; *reason = 8; }
    }
    if (e->st.player == WHITE) e->move_count++;                                         /* 291-292 */
    *reward = rw;
    *done = e->done;
    return 0;
}

/* The single-board env's primitive ops (the device's gc_env_single_call, k_single): one
 * ChessEnvV2.step() (chess_v2.py:219-294) split where a host opponent policy must see the
 * move list.  op 0 reset (183-206, no opening), 1 the agent's step up to the opponent's turn
 * (flags bit 0: an opponent follows, so the move count waits for it), 2 the opponent's reply,
 * 3 the opponent's opening (208-216), 4 nothing.  out = {status (1: both kings checked, the
 * engine raises, nothing changes), reward, done, reason} with the batched step's reasons. */
int oracle_single_op(void *h, int op, int action, int flags, int *out) {
    OEnv *e = (OEnv *)h;
    int status = 0, reward = 0, done = 0, reason = 0, mr = 0, rep = 0;
    if (op == 0) {
        int opp = e->opp;
        e->opp = 0;
        o_env_reset(e);
        e->opp = opp;
    } else if (op == 1) {
        int valid = 0;
        for (int k = 0; k < e->nmoves; k++) if (e->moves[k] == action) { valid = 1; break; }
        if (!valid) { reward = -10; done = e->done; reason = 6; }                          /* 239-242 */
        else if (e->done) { done = 1; reason = 7; }                                        /* 245-251 */
        else if (e->move_count > 149) { done = 1; reason = 3; }                            /* 252-258 */
        else if (env_player_move(e, action, &mr, &rep) == 1) status = 1;                    /* lib.rs:1442 */
        else {
            reward = -10 + mr;                                                              /* 261-264 */
            e->done = rep;
            if (rep) { done = 1; reason = 2; }
            int chk = e->st.player == WHITE ? e->st.wchk : e->st.bchk;
            if (e->nmoves == 0 && chk) { e->done = 1; done = 1; reward += 100; reason = 1; } /* 269-272 */
            if (!done && !(flags & 1) && e->st.player == WHITE) e->move_count++;           /* 291-292 */
        }
    } else if (op == 2) {                                                                   /* 275-292 */
        if (env_player_move(e, action, &mr, &rep) == 1) status = 1;
        else {
            reward = -mr;
            e->done = rep;
            if (rep) { done = 1; reason = 2; }
            int chk = e->st.player == WHITE ? e->st.wchk : e->st.bchk;
            if (e->nmoves == 0 && chk) { e->done = 1; done = 1; reward -= 100; reason = 8; }
            if (e->st.player == WHITE) e->move_count++;
        }
    } else if (op == 3) {                                                                   /* 208-216 */
        if (env_player_move(e, action, &mr, &rep) == 1) status = 1;
        else { e->done = 0; e->move_count = 1; }
    }
    out[0] = status; out[1] = reward; out[2] = done; out[3] = reason;
    return status;
}

/* ---- Philox4x32-10 (Salmon et al. 2011) for the on-device random policy --- */
static void philox(uint32_t c[4], const uint32_t k0in, const uint32_t k1in, uint32_t out[4]) {
    uint32_t k0 = k0in, k1 = k1in;
    uint32_t x0 = c[0], x1 = c[1], x2 = c[2], x3 = c[3];
    for (int i = 0; i < 10; i++) {
        uint64_t p0 = (uint64_t)0xD2511F53u * x0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * x2;
        uint32_t y0 = (uint32_t)(p1 >> 32) ^ x1 ^ k0;
        uint32_t y1 = (uint32_t)p1;
        uint32_t y2 = (uint32_t)(p0 >> 32) ^ x3 ^ k1;
        uint32_t y3 = (uint32_t)p0;
        x0 = y0; x1 = y1; x2 = y2; x3 = y3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = x0; out[1] = x1; out[2] = x2; out[3] = x3;
}
/* policy draw: uniform index in [0,n) for (seed, board, draw#) */
uint32_t oracle_policy_index(uint64_t seed, uint32_t board, uint32_t draw, uint32_t n) {
    uint32_t c[4] = {board, draw, 0x5EEDu, 0u}, o[4];
    philox(c, (uint32_t)seed, (uint32_t)(seed >> 32), o);
    return (uint32_t)(((uint64_t)o[0] * n) >> 32);
}

/* Rank k -> the k-th legal action in ascending action id: the order of a legal-action mask,
 * which the device API step's `pick` output follows (the policy itself ranks in move-set
 * order, kth_in_set_order).  Any fixed bijection gives the same uniform policy. */
static int kth_in_action_order(const uint16_t *moves, int n, int k) {
    uint16_t tmp[MAXMOVES];
    for (int i = 0; i < n; i++) {  /* insertion sort: lists are short */
        uint16_t v = moves[i];
        int j = i;
        while (j > 0 && tmp[j - 1] > v) { tmp[j] = tmp[j - 1]; j--; }
        tmp[j] = v;
    }
    return tmp[k];
}

/* The self-play policy's order (the device's gc_core.h sw_gen / sw_select, restated from the
 * move's geometry): a legal move belongs to one of 28 sets -- pawn single push, double push,
 * capture toward col+1, toward col-1; the eight knight jumps; rooks / queens by direction
 * (row-1, row+1, col+1, col-1); bishops / queens by direction (row-1 col+1, row-1 col-1,
 * row+1 col+1, row+1 col-1); the eight king steps -- ordered by set, then by target square;
 * castles last, queen side first.  Any fixed bijection gives the same uniform policy; this
 * is the one the device enumerates without a per-piece loop. */
static int sgn(int x) { return (x > 0) - (x < 0); }
static int set_key(const int8_t *b, int a) {
    static const int8_t kn[8][2] = {{2, -1}, {2, 1}, {-2, -1}, {-2, 1}, {1, -2}, {1, 2}, {-1, -2}, {-1, 2}};
    static const int8_t kg[8][2] = {{-1, 0}, {1, 0}, {0, -1}, {0, 1}, {-1, -1}, {-1, 1}, {1, -1}, {1, 1}};
    static const int8_t sl[8][2] = {{-1, 0}, {1, 0}, {0, 1}, {0, -1}, {-1, 1}, {-1, -1}, {1, 1}, {1, -1}};
    if (a >= 4096) return 28 * 64 + ((a == 4097 || a == 4099) ? 0 : 1);  /* QS (4097 / 4099), KS */
    int f = a >> 6, t = a & 63, dr = (t >> 3) - (f >> 3), dc = (t & 7) - (f & 7);
    int ty = b[f] < 0 ? -b[f] : b[f], set = -1;
    if (ty == PAWN) {
        set = dc == 0 ? ((dr == 1 || dr == -1) ? 0 : 1) : (dc > 0 ? 2 : 3);
    } else if (ty == KNIGHT) {
        for (int i = 0; i < 8; i++) if (kn[i][0] == dr && kn[i][1] == dc) set = 4 + i;
    } else if (ty == KING) {
        for (int i = 0; i < 8; i++) if (kg[i][0] == dr && kg[i][1] == dc) set = 20 + i;
    } else {  /* Q, R, B: the direction of the ray */
        for (int i = 0; i < 8; i++) if (sl[i][0] == sgn(dr) && sl[i][1] == sgn(dc)) set = 12 + i;
    }
    return set * 64 + t;
}
static int kth_in_set_order(const int8_t *b, const uint16_t *moves, int n, int k) {
    uint16_t tmp[MAXMOVES];
    int key[MAXMOVES];
    for (int i = 0; i < n; i++) {  /* insertion sort by key: lists are short */
        uint16_t v = moves[i];
        int kv = set_key(b, v), j = i;
        while (j > 0 && key[j - 1] > kv) { tmp[j] = tmp[j - 1]; key[j] = key[j - 1]; j--; }
        tmp[j] = v;
        key[j] = kv;
    }
    return tmp[k];
}

/* Random self-play rollout of one board (the test_benchmark.py driver shape, auto-reset):
 * at each ply: if no legal moves -> episode ends (driver `break`), reset, no step counted;
 * else action = moves[policy_index(...)], step; if done -> reset.
 * Trajectory out (optional, length plies): action, reward, done, reason per ply.
 * Counters: steps taken; episodes by reason [0 none,1 mate,2 rep,3 cap,4 stalemate,5 error]. */
typedef struct { uint64_t steps, reward_sum, ends[6]; int max_win; } OStats; /* ends[0] unused; max_win: longest window */

static int stats_slot(int reason) { return reason == 8 ? 1 : (reason == 9 ? 4 : (reason == 10 ? 5 : reason)); }

static void rollout_board(const int8_t *init, uint64_t seed, uint32_t board, int plies, int opp, int agent_black,
                          int order, int16_t *tr_action, int16_t *tr_reward, uint8_t *tr_done, uint8_t *tr_reason,
                          int8_t *final_board, uint8_t *final_meta, uint32_t *final_draw, OStats *st) {
    OEnv e;
    memset(&e, 0, sizeof(e));
    memcpy(e.init, init, 64);
    e.opp = opp; e.agent_black = agent_black; e.seed = seed; e.board = board; e.draw = 0;
    e.set_order = order < 0 ? 1 : order;
    o_env_reset(&e);
    for (int p = 0; p < plies; p++) {
        int action = -1, rw = 0, dn = 0, reason = 0;
        if (e.nmoves == 0) {
            /* test_benchmark.py:22-24: driver breaks on an empty move list */
            reason = 4;
            st->ends[4]++;
            o_env_reset(&e);
        } else {
            action = env_policy_pick(&e);
            int rc = o_env_step(&e, action, &rw, &dn, &reason);
            st->steps++;
            st->reward_sum += (uint64_t)(int64_t)rw;
            if (rc == 1) { reason = 5; dn = 1; }
            if (e.win > st->max_win) st->max_win = e.win;
            if (dn) { st->ends[stats_slot(reason)]++; o_env_reset(&e); }
        }
        if (tr_action) {
            tr_action[p] = (int16_t)action; tr_reward[p] = (int16_t)rw;
            tr_done[p] = (uint8_t)dn; tr_reason[p] = (uint8_t)reason;
        }
    }
    if (final_board) {
        memcpy(final_board, e.st.b, 64);
        final_meta[0] = e.st.player == WHITE;
        final_meta[1] = e.st.wkc; final_meta[2] = e.st.wqc; final_meta[3] = e.st.bkc; final_meta[4] = e.st.bqc;
        final_meta[5] = e.st.wchk; final_meta[6] = e.st.bchk; final_meta[7] = (uint8_t)e.move_count;
    }
    if (final_draw) *final_draw = e.draw;
    free(e.saved);
    free(e.cnt);
}

/* Single-board trajectory for parity tests. */
void oracle_rollout_trace(const int8_t *init, uint64_t seed, uint32_t board, int plies,
                          int16_t *tr_action, int16_t *tr_reward, uint8_t *tr_done, uint8_t *tr_reason,
                          int8_t *final_board, uint8_t *final_meta, uint64_t *stats8) {
    OStats st;
    memset(&st, 0, sizeof(st));
    uint32_t draw;
    rollout_board(init, seed, board, plies, 0, 0, -1, tr_action, tr_reward, tr_done, tr_reason, final_board, final_meta, &draw, &st);
    if (stats8) { stats8[0] = st.steps; stats8[1] = st.reward_sum; for (int i = 0; i < 6; i++) stats8[2 + i] = st.ends[i]; }
}

/* Multi-threaded batch rollout = CPU baseline (boards sharded across pthreads). */
typedef struct { const int8_t *init; uint64_t seed; uint32_t b0, b1; int plies, opp, agent_black; OStats st; } Job;
static void *job_run(void *arg) {
    Job *j = (Job *)arg;
    memset(&j->st, 0, sizeof(j->st));
    for (uint32_t b = j->b0; b < j->b1; b++)
        rollout_board(j->init, j->seed, b, j->plies, j->opp, j->agent_black, -1, NULL, NULL, NULL, NULL, NULL, NULL, NULL, &j->st);
    return NULL;
}
void oracle_rollout_batch2(const int8_t *init, uint64_t seed, uint32_t b_begin, uint32_t n_boards, int plies,
                           int opp, int agent_white, int threads, uint64_t *stats8) {
    int agent_black = !agent_white;
    if (threads < 1) threads = 1;
    Job *jobs = (Job *)calloc((size_t)threads, sizeof(Job));
    pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    for (int t = 0; t < threads; t++) {
        jobs[t].init = init; jobs[t].seed = seed; jobs[t].plies = plies; jobs[t].opp = opp; jobs[t].agent_black = agent_black;
        jobs[t].b0 = b_begin + (uint32_t)((uint64_t)n_boards * t / threads);
        jobs[t].b1 = b_begin + (uint32_t)((uint64_t)n_boards * (t + 1) / threads);
        pthread_create(&th[t], NULL, job_run, &jobs[t]);
    }
    memset(stats8, 0, 8 * sizeof(uint64_t));
    for (int t = 0; t < threads; t++) {
        pthread_join(th[t], NULL);
        stats8[0] += jobs[t].st.steps; stats8[1] += jobs[t].st.reward_sum;
        for (int i = 0; i < 6; i++) stats8[2 + i] += jobs[t].st.ends[i];
    }
    free(jobs);
    free(th);
}

void oracle_rollout_batch(const int8_t *init, uint64_t seed, uint32_t b_begin, uint32_t n_boards, int plies,
                          int threads, uint64_t *stats8) {
    oracle_rollout_batch2(init, seed, b_begin, n_boards, plies, 0, 1, threads, stats8);
}

/* Full-width trajectory digests: one 64-bit digest per board of its whole
 * rollout_board trajectory -- every ply's outputs packed as the device's trace word (action i16 |
 * reward i16 << 16 | done << 32 | reason << 40, gymchess.hip trace_word), folded in ply order by
 * d = (d ^ w) * FNV_PRIME, then the final state's 64 board bytes as eight little-endian words and
 * its 8 meta bytes as one.  Boards handed out across pthreads. */
#define DIGEST_PRIME 0x100000001B3ull
static uint64_t digest_fold(uint64_t d, uint64_t w) { return (d ^ w) * DIGEST_PRIME; }
uint64_t oracle_trace_word(int action, int reward, int done, int reason) {
    return (uint64_t)(uint16_t)(int16_t)action | ((uint64_t)(uint16_t)(int16_t)reward << 16) |
           ((uint64_t)(done & 0xFF) << 32) | ((uint64_t)(reason & 0xFF) << 40);
}
typedef struct {
    const int8_t *init; uint64_t seed; int plies, opp, agent_black; uint32_t b_begin, n; atomic_uint *next;
    uint64_t *out;
} DJob;
static void *djob_run(void *arg) {
    DJob *j = (DJob *)arg;
    int16_t *a = (int16_t *)malloc((size_t)j->plies * 2), *r = (int16_t *)malloc((size_t)j->plies * 2);
    uint8_t *dn = (uint8_t *)malloc((size_t)j->plies), *why = (uint8_t *)malloc((size_t)j->plies);
    for (;;) {
        uint32_t k = atomic_fetch_add(j->next, 1u);
        if (k >= j->n) break;
        OStats st;
        memset(&st, 0, sizeof(st));
        int8_t fb[64];
        uint8_t fm[8];
        uint32_t draw;
        rollout_board(j->init, j->seed, j->b_begin + k, j->plies, j->opp, j->agent_black, -1, a, r, dn, why, fb, fm, &draw,
                      &st);
        uint64_t d = 0, w;
        for (int p = 0; p < j->plies; p++) d = digest_fold(d, oracle_trace_word(a[p], r[p], dn[p], why[p]));
        for (int q = 0; q < 8; q++) { memcpy(&w, fb + 8 * q, 8); d = digest_fold(d, w); }
        memcpy(&w, fm, 8);
        j->out[k] = digest_fold(d, w);
    }
    free(a); free(r); free(dn); free(why);
    return NULL;
}
void oracle_rollout_digests(const int8_t *init, uint64_t seed, uint32_t b_begin, uint32_t n_boards, int plies, int opp,
                            int agent_white, int threads, uint64_t *out) {
    if (threads < 1) threads = 1;
    atomic_uint next;
    atomic_init(&next, 0u);
    DJob *jobs = (DJob *)calloc((size_t)threads, sizeof(DJob));
    pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    for (int t = 0; t < threads; t++) {
        jobs[t] = (DJob){init, seed, plies, opp, !agent_white, b_begin, n_boards, &next, out};
        pthread_create(&th[t], NULL, djob_run, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    free(jobs);
    free(th);
}

/* Trajectory with an opponent mode (0 none, 1 random) and agent colour; order -1 or 1: the
 * policy's move-set order, 0: action-id order (the API step's `pick` output). */
void oracle_rollout_trace3(const int8_t *init, uint64_t seed, uint32_t board, int plies, int opp, int agent_white,
                           int order, int16_t *tr_action, int16_t *tr_reward, uint8_t *tr_done, uint8_t *tr_reason,
                           int8_t *final_board, uint8_t *final_meta, uint64_t *stats8) {
    OStats st;
    memset(&st, 0, sizeof(st));
    uint32_t draw;
    rollout_board(init, seed, board, plies, opp, !agent_white, order, tr_action, tr_reward, tr_done, tr_reason, final_board,
                  final_meta, &draw, &st);
    if (stats8) { stats8[0] = st.steps; stats8[1] = st.reward_sum; for (int i = 0; i < 6; i++) stats8[2 + i] = st.ends[i]; }
}

/* the longest 3-fold window (distinct pre-move boards since the last pawn move / capture)
 * along the same trajectory as oracle_rollout_trace3 */
int oracle_rollout_max_window(const int8_t *init, uint64_t seed, uint32_t board, int plies, int opp, int agent_white) {
    OStats st;
    memset(&st, 0, sizeof(st));
    rollout_board(init, seed, board, plies, opp, !agent_white, -1, NULL, NULL, NULL, NULL, NULL, NULL, NULL, &st);
    return st.max_win;
}

void oracle_rollout_trace2(const int8_t *init, uint64_t seed, uint32_t board, int plies, int opp, int agent_white,
                           int16_t *tr_action, int16_t *tr_reward, uint8_t *tr_done, uint8_t *tr_reason,
                           int8_t *final_board, uint8_t *final_meta, uint64_t *stats8) {
    oracle_rollout_trace3(init, seed, board, plies, opp, agent_white, -1, tr_action, tr_reward, tr_done, tr_reason,
                          final_board, final_meta, stats8);
}

/* Multi-threaded perft over many roots (CPU baseline for perft configs).  Roots are handed
 * out one at a time from a shared counter: subtree sizes vary by 10x between mid-game roots,
 * so a static split leaves most threads idle behind the largest ones. */
typedef struct { const int8_t *boards; const uint8_t *metas; int depth; uint32_t n; atomic_uint *next; uint64_t *out; } PJob;
static void *pjob_run(void *arg) {
    PJob *j = (PJob *)arg;
    for (;;) {
        uint32_t b = atomic_fetch_add(j->next, 1u);
        if (b >= j->n) break;
        j->out[b] = oracle_perft(j->boards + 64 * (size_t)b, j->metas + 8 * (size_t)b, j->depth);
    }
    return NULL;
}
void oracle_perft_batch(const int8_t *boards, const uint8_t *metas, uint32_t n, int depth, int threads, uint64_t *out) {
    if (threads < 1) threads = 1;
    atomic_uint next;
    atomic_init(&next, 0u);
    PJob *jobs = (PJob *)calloc((size_t)threads, sizeof(PJob));
    pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    for (int t = 0; t < threads; t++) {
        jobs[t].boards = boards; jobs[t].metas = metas; jobs[t].depth = depth; jobs[t].out = out;
        jobs[t].n = n; jobs[t].next = &next;
        pthread_create(&th[t], NULL, pjob_run, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    free(jobs);
    free(th);
}

/* Env handle API for step-by-step trace tests (Python drives actions). */
void *oracle_env_new2(const int8_t *init, int opp, int agent_white, uint64_t seed, uint32_t board) {
    OEnv *e = (OEnv *)calloc(1, sizeof(OEnv));
    memcpy(e->init, init, 64);
    e->opp = opp; e->agent_black = !agent_white; e->seed = seed; e->board = board;
    e->set_order = 1;
    o_env_reset(e);
    return e;
}
void *oracle_env_new(const int8_t *init) { return oracle_env_new2(init, 0, 1, 0, 0); }
uint32_t oracle_env_draw(void *h) { return ((OEnv *)h)->draw; }
/* the self-play driver's pick for the side to move (same stream as the opponent's); -1 if none */
int oracle_env_pick(void *h) { OEnv *e = (OEnv *)h; return e->nmoves ? env_policy_pick(e) : -1; }
void oracle_env_free(void *h) { OEnv *e = (OEnv *)h; free(e->saved); free(e->cnt); free(e); }
void oracle_env_reset(void *h) { o_env_reset((OEnv *)h); }
int oracle_env_step(void *h, int action, int *reward, int *done, int *reason) { return o_env_step((OEnv *)h, action, reward, done, reason); }
int oracle_env_moves(void *h, uint16_t *out, int cap) {
    OEnv *e = (OEnv *)h;
    for (int k = 0; k < e->nmoves && k < cap; k++) out[k] = e->moves[k];
    return e->nmoves;
}
void oracle_env_state(void *h, int8_t *board, uint8_t *meta) {
    OEnv *e = (OEnv *)h;
    memcpy(board, e->st.b, 64);
    meta[0] = e->st.player == WHITE;
    meta[1] = e->st.wkc; meta[2] = e->st.wqc; meta[3] = e->st.bkc; meta[4] = e->st.bqc;
    meta[5] = e->st.wchk; meta[6] = e->st.bchk; meta[7] = (uint8_t)e->move_count;
}
int oracle_env_done(void *h) { return ((OEnv *)h)->done; }
/* the state setter (chess_v2.py:315-323): board, the four rights, the two check flags;
 * current_player, move_count, done and saved_boards stay.  The move list is that of the new
 * board (the device's SET does the same; the single-board env keeps the reference's stale
 * possible_moves on the host). */
void oracle_env_set_board(void *h, const int8_t *board, const uint8_t *flags6) {
    OEnv *e = (OEnv *)h;
    memcpy(e->st.b, board, 64);
    e->st.wkc = flags6[0] != 0; e->st.wqc = flags6[1] != 0; e->st.bkc = flags6[2] != 0; e->st.bqc = flags6[3] != 0;
    e->st.wchk = flags6[4] != 0; e->st.bchk = flags6[5] != 0;
    OState s;
    env_engine_state(e, &s);
    e->nmoves = o_get_possible_moves(&s, e->st.player, 0, e->moves, MAXMOVES);
}
/* distinct pre-move boards since the last pawn move / capture (the device's window length,
 * which its per-board table holds up to hist_cap and its spill table beyond) */
int oracle_env_window(void *h) { return ((OEnv *)h)->win; }
