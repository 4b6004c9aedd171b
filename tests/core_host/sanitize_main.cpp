// TEST INFRASTRUCTURE ONLY: the host build of the product's bitboard core (core_host.cpp,
// i.e. gc_core.h / gc_env.h / gc_fide.h) linked with the C oracle under AddressSanitizer and
// UndefinedBehaviorSanitizer (SURVEY.md §5 "Race detection/sanitizers"; GPU ASan is not
// available on this pool, so the device code is sanitized in its host form).  A seeded
// differential run: random positions (also kingless / several kings / pawns on back ranks)
// -> ordered move lists (legal and attack mode), castle lists, update_state, next_state of
// every legal move, perft(2); whole self-play trajectories with and without the random
// opponent; FIDE perft from the start position.  Exit 0 = no mismatch and no sanitizer report
// (sanitizers abort: -fno-sanitize-recover=all).
#include "core_host.cpp"

#include <cstdio>
#include <cstdlib>

extern "C" {
int oracle_get_possible_moves(const int8_t* board, const uint8_t* meta, int player_white, int attack, uint16_t* out,
                              int cap);
int oracle_get_castle_moves(const int8_t* board, const uint8_t* meta, int player_white, uint16_t* out);
int oracle_next_state(const int8_t* board, const uint8_t* meta, int player_white, int action, int8_t* ob,
                      uint8_t* om, int* reward);
void oracle_update_state(const int8_t* board, const uint8_t* meta, int8_t* ob, uint8_t* om);
uint64_t oracle_perft(const int8_t* board, const uint8_t* meta, int depth);
void oracle_rollout_trace2(const int8_t* init, uint64_t seed, uint32_t board, int plies, int opp, int agent_white,
                           int16_t* tr_action, int16_t* tr_reward, uint8_t* tr_done, uint8_t* tr_reason,
                           int8_t* final_board, uint8_t* final_meta, uint64_t* stats8);
}

static uint64_t rng_state = 0x5EED5EEDull;
static uint32_t rnd(uint32_t n) {
    rng_state = rng_state * 6364136223846793005ull + 1442695040888963407ull;
    return (uint32_t)((rng_state >> 33) % n);
}

static int fails = 0;
#define CHECK(c, ...)                        \
    do {                                     \
        if (!(c)) {                          \
            fprintf(stderr, __VA_ARGS__);    \
            fputc('\n', stderr);             \
            if (++fails > 20) exit(1);       \
        }                                    \
    } while (0)

static void random_position(int8_t* b, uint8_t* m) {
    static const int8_t ids[] = {2, 3, 4, 5, 6, 6, 6, -2, -3, -4, -5, -6, -6, -6};
    memset(b, 0, 64);
    int k = 2 + (int)rnd(24);
    for (int j = 0; j < k; j++) b[rnd(64)] = ids[rnd(14)];
    int mode = (int)rnd(10);
    if (mode != 1) b[rnd(64)] = 1;
    if (mode != 2) b[rnd(64)] = -1;
    if (mode == 3) b[rnd(64)] = rnd(2) ? 1 : -1;
    m[0] = (uint8_t)rnd(2);
    for (int j = 1; j < 5; j++) m[j] = (uint8_t)rnd(2);
    m[5] = m[6] = m[7] = 0;
}

int main(int argc, char** argv) {
    int positions = argc > 1 ? atoi(argv[1]) : 300;
    int8_t b[64], ob[64], rb[64];
    uint8_t m[8], om[8], rm[8];
    uint16_t hl[512], rl[512];
    for (int t = 0; t < positions; t++) {
        random_position(b, m);
        for (int attack = 0; attack < 2; attack++)
            for (int white = 0; white < 2; white++) {
                int nh = host_list(b, m, white, attack, hl, 512);
                int nr = oracle_get_possible_moves(b, m, white, attack, rl, 512);
                CHECK(nh == nr && memcmp(hl, rl, 2 * (size_t)nh) == 0, "list mismatch pos %d attack %d white %d", t,
                      attack, white);
            }
        host_update_state(b, m, ob, om);
        oracle_update_state(b, m, rb, rm);
        CHECK(memcmp(ob, rb, 64) == 0 && memcmp(om, rm, 7) == 0, "update_state mismatch pos %d", t);
        int n = oracle_get_possible_moves(b, m, m[0], 0, rl, 512);
        for (int k = 0; k < n; k++) {
            int hr = 0, rr = 0;
            int hc = host_next_state(b, m, m[0], rl[k], ob, om, &hr);
            int rc = oracle_next_state(b, m, m[0], rl[k], rb, rm, &rr);
            CHECK(hc == rc && hr == rr && memcmp(ob, rb, 64) == 0 && memcmp(om, rm, 7) == 0,
                  "next_state mismatch pos %d move %d", t, rl[k]);
        }
        CHECK(host_perft(b, m, 2) == oracle_perft(b, m, 2), "perft(2) mismatch pos %d", t);
    }
    static const int8_t start[64] = {-3, -5, -4, -2, -1, -4, -5, -3, -6, -6, -6, -6, -6, -6, -6, -6,
                                     0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,
                                     0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,
                                     6,  6,  6,  6,  6,  6,  6,  6,  3,  5,  4,  2,  1,  4,  5,  3};
    const int plies = 400;
    std::vector<int16_t> ha(plies), hr(plies), ra(plies), rr(plies);
    std::vector<uint8_t> hd(plies), hq(plies), rd(plies), rq(plies);
    uint64_t hs[8], rs[8];
    for (int opp = 0; opp < 2; opp++)
        for (uint32_t board = 0; board < 12; board++) {
            int aw = opp ? (int)(board & 1) : 1;
            host_rollout_trace2(start, 0xABCD, board, plies, opp, aw, ha.data(), hr.data(), hd.data(), hq.data(), ob,
                                om, hs);
            oracle_rollout_trace2(start, 0xABCD, board, plies, opp, aw, ra.data(), rr.data(), rd.data(), rq.data(), rb,
                                  rm, rs);
            CHECK(ha == ra && hr == rr && hd == rd && hq == rq && memcmp(ob, rb, 64) == 0 && memcmp(hs, rs, 64) == 0,
                  "rollout mismatch opp %d board %u", opp, board);
        }
    uint8_t sm[8] = {1, 1, 1, 1, 1, 0, 0, 0};
    CHECK(host_fide_perft(start, sm, 3) == 8902, "FIDE perft(3) of the start position");
    printf("sanitized differential run: %d positions, 24 rollouts x %d plies, fails %d\n", positions, plies, fails);
    return fails ? 1 : 0;
}
