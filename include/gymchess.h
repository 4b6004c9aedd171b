/* gymchess.h -- C-ABI of libgymchess.so, the MI355X-native drop-in for the gym-chess
 * hot path (reference: /root/reference, bobu36000/gym-chess).
 *
 * Plain pointers and sizes only.  All host buffers are caller-owned; device memory is
 * owned by the handles.  Every function returns 0 on success, non-zero on failure with a
 * message in gc_last_error() (per calling thread).  One handle per host thread/stream.
 *
 * Conventions (identical to the reference):
 *   board   int8[64], sq = row*8 + col, row 0 = rank 8 (lib.rs:1235-1238);
 *           ids +-1..6 = K,Q,R,B,N,P, positive = WHITE (lib.rs:11-17, 41-50)
 *   meta    uint8[8] = {white_to_move, white_king_castle_is_possible,
 *           white_queen_castle_is_possible, black_king_castle_is_possible,
 *           black_queen_castle_is_possible, white_king_is_checked,
 *           black_king_is_checked, move_count}  (the state dict, lib.rs:355-395)
 *   action  uint16: from*64 + to; 4096 CASTLE_KING_SIDE_WHITE, 4097 ..._QUEEN_SIDE_WHITE,
 *           4098 ..._KING_SIDE_BLACK, 4099 ..._QUEEN_SIDE_BLACK, 4100 RESIGN
 *           (chess_v2.py:492-532); 0xFFFF = "no legal move" in policy buffers.
 */
#ifndef GYMCHESS_H
#define GYMCHESS_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GC_ABI_VERSION 1

const char* gc_last_error(void);
int gc_version(void);
/* "gymchess-src-hash:<hex>": the sha256 prefix of the sources and compile flags this library
 * was built from (the Python loader refuses a library whose hash differs from its sources') */
const char* gc_build_hash(void);
int gc_get_device_count(int* n);

/* ---------------------------------------------------------------------------------
 * Stateless engine: batched form of the reference FFI class `ChessEngine`
 * (#[pyclass] at /root/reference/src/lib.rs:1412-1512, bound in Python at
 * gym_chess/__init__.py:1, used at chess_v2.py:146, 204, 419, 579, 590).
 * ------------------------------------------------------------------------------- */
typedef struct gc_engine gc_engine;
int gc_engine_create(int device, gc_engine** out);
int gc_engine_destroy(gc_engine* e);

/* replaces ChessEngine.get_possible_moves(state, player, attack=False) (lib.rs:1454-1480):
 * per board the ordered action list (normal moves in reference order, then castles QS, KS;
 * attack != 0: attack-mode moves, no castles).  moves is n*cap; counts[i] may exceed cap
 * (list truncated). player_white[i] is the `player` argument. */
int gc_engine_get_possible_moves(gc_engine* e, int n, const int8_t* boards, const uint8_t* meta,
                                 const uint8_t* player_white, int attack, uint16_t* moves, int cap,
                                 int32_t* counts);
/* replaces ChessEngine.get_castle_moves(state, player) (lib.rs:1482-1500); moves is n*2 */
int gc_engine_get_castle_moves(gc_engine* e, int n, const int8_t* boards, const uint8_t* meta,
                               const uint8_t* player_white, uint16_t* moves, int32_t* counts);
/* replaces ChessEngine.next_state(state, player, move) (lib.rs:1422-1452): move, reward,
 * update_state.  status[i]: 0 ok; 1 both kings checked (the reference sets a Python
 * exception); -1 empty from-square (the reference panics); -2 bad action. */
int gc_engine_next_state(gc_engine* e, int n, const int8_t* boards, const uint8_t* meta,
                         const uint8_t* player_white, const uint16_t* actions, int8_t* out_boards,
                         uint8_t* out_meta, int32_t* rewards, int32_t* status);
/* replaces ChessEngine.update_state(state) (lib.rs:1502-1511) */
int gc_engine_update_state(gc_engine* e, int n, const int8_t* boards, const uint8_t* meta,
                           int8_t* out_boards, uint8_t* out_meta);
/* perft by composition of get_all_possible_moves and next_state; the side
 * to move is meta[0]. depth in [0, 8]; any n (levels too large for HBM are expanded one
 * chunk of parents at a time, sizes are 64-bit). */
int gc_engine_perft(gc_engine* e, int n, const int8_t* boards, const uint8_t* meta, int depth,
                    uint64_t* nodes);
/* diagnostics: how many times each perft leaf pass ran in this process, out4 = {split
 * (depth-3 subtrees split to depth-2, sorted), sorted (subtrees by move count), small
 * (unsorted nested loops), fide} */
int gc_perft_path_counts(uint64_t* out4);
/* diagnostics: the split pass's leaf kernel (k_perft2_rec / k_perft2_val, one lane = one
 * depth-2 subtree) in this process -- launches, subtrees counted and summed kernel time (HIP
 * events on its stream) */
int gc_perft_leaf_stats(uint64_t* launches, uint64_t* subtrees, double* kernel_ms);
/* diagnostics: the split pass's depth-2 roots made (records) and counted (one per distinct
 * position of a chunk when the transposition pass runs, GC_PERFT_DEDUP != 0) in this process */
int gc_perft_dedup_stats(uint64_t* records, uint64_t* counted);
/* Rules of every later call on this engine (not in the reference):
 * 0 = the reference's (default, lib.rs), 1 = FIDE (gym-chess_amd/csrc/gc_fide.h: en passant,
 * promotion, per-side castling through unattacked squares, no king captures).  Under FIDE
 * rules meta[7] is the en-passant FILE + 1 (0 = none) on input and output; move lists hold
 * each promotion once (as a queen promotion) in ascending action id, castles last; perft
 * counts the four promotion pieces. */
int gc_engine_set_rules(gc_engine* e, int rules);

/* ---------------------------------------------------------------------------------
 * Batched env: N independent ChessEnvV2(opponent="none") boards resident on one device
 * (chess_v2.py:132-602 reset()/step()/possible_moves).
 * ------------------------------------------------------------------------------- */
typedef struct gc_env gc_env;
/* initial_board: int8[64] or NULL for DEFAULT_BOARD (chess_v2.py:98-107) */
int gc_env_create(int device, int n_boards, uint64_t seed, const int8_t* initial_board, gc_env** out);
int gc_env_destroy(gc_env* e);
int gc_env_num_boards(gc_env* e);
/* Opponent mode (replaces ChessEnvV2(player_color, opponent), chess_v2.py:133-181):
 * opponent 0 = "none", 1 = "random" -- the device policy replies inside every step()
 * (chess_v2.py:275-292: -opp_reward, -100 when the agent is then mated); agent_white 0 =
 * player_color BLACK (the opponent opens at every reset, chess_v2.py:208-216; requires
 * opponent 1).  Resets every board.  A callable opponent = opponent 0 with the caller
 * stepping both sides. */
int gc_env_set_opponent(gc_env* e, int opponent, int agent_white);
/* ---- single-board env ops (the ChessEnvV2-shaped env gym_chess_amd.single.ChessEnv,
 * whose opponent policy is a host callable: "random" draws from numpy's global generator,
 * chess_v2.py:116-127).  One ChessEnvV2.step() (chess_v2.py:219-294) is split where the
 * policy must see the move list: op 1 AGENT runs the agent's step up to the opponent's turn
 * (validation 239-242, the done / move-cap early returns 245-258, player_move with the
 * 3-fold count of the pre-move board 393-412, mate +100 269-272, and -- flags bit 0 clear,
 * no opponent follows -- the move-count rule 291-292); op 2 REPLY the opponent's
 * player_move (-its capture value, -100 if the agent is mated, the move-count rule); op 0
 * RESET reset() up to the BLACK opening (183-206); op 3 OPEN the opponent's opening move
 * (208-216: its 3-fold verdict discarded, move_count 1); op 4 SYNC no change.  Each op is
 * one launch on board `board` of the env; the result lands in a host-mapped record owned by
 * the env (*rec, valid until the next call): status 1 = the engine's both-kings-checked error
 * (lib.rs:1442-1446; nothing changed), the op's reward / done / reason (the batched step's
 * reason codes), the state and the move list of the side to move in reference order
 * (lib.rs:460-563, castles QS then KS).  gc_env_single_setup(agent_white = 0) gives a BLACK
 * agent's board the uncapped window (its move_count never advances, 291-292). */
#define GC_SINGLE_MOVES_CAP 320
typedef struct {
    int32_t status, reward;
    uint8_t done, reason, env_done, white_to_move;
    uint8_t rights[4];   /* wkc wqc bkc bqc */
    uint8_t checked[2];  /* white, black */
    uint16_t move_count;
    int32_t nmoves;      /* legal moves of the side to move (moves holds the first 320) */
    int8_t board[64];
    uint16_t moves[GC_SINGLE_MOVES_CAP];
} gc_single_record;
int gc_env_single_setup(gc_env* e, int agent_white);
int gc_env_single_call(gc_env* e, int board, int op, int action, int flags, const gc_single_record** rec);
/* diagnostic: the single-board server's last op by segment, in 10 ns ticks: {the request's read
 * and validation, the ply, the move list, the outcome and stores, the record's copy to host
 * memory, the wait for the request} */
int gc_env_single_stamps(gc_env* e, uint32_t* out6);
/* the env's state setter (chess_v2.py:315-323) on board `board`: its pieces (int8[64]) and
 * flags6 = {wkc, wqc, bkc, bqc, white_checked, black_checked}; the side to move, move_count,
 * done and the 3-fold window stay.  *rec as gc_env_single_call (the new position's list). */
int gc_env_single_set(gc_env* e, int board, const int8_t* board64, const uint8_t* flags6, const gc_single_record** rec);
/* The live 3-fold window of one board (the boards since its last pawn move / capture and
 * their pre-move occurrence counts; chess_v2.py's saved_boards minus the boards that can no
 * longer recur): up to cap boards int8[64] and counts; *n = the window's length. */
int gc_env_window_boards(gc_env* e, int board, int8_t* boards, uint8_t* counts, int cap, int* n);
/* reset() (chess_v2.py:183-217) of the boards with mask[i] != 0 (mask NULL = all) */
int gc_env_reset(gc_env* e, const uint8_t* mask);
/* step(action) (chess_v2.py:219-294) for every board; host buffers of n entries.
 * reason[i]: 0 none, 1 mate (+100), 2 3-fold repetition, 3 move cap, 5 both kings checked
 * (reference raises; state unchanged), 6 invalid action (-10), 7 step after done,
 * 8 agent mated by the opponent's reply (-100), 9 the opponent has no legal reply (the
 * reference's random policy returns "resign", which maps to no action and raises). */
int gc_env_step(gc_env* e, const uint16_t* actions, int32_t* reward, uint8_t* done, uint8_t* reason);
/* step(action) with DEVICE buffers, for a policy that lives on the GPU (chess_v2.py:219-294
 * + the rebuilt possible_actions, 333-335): d_actions[n] in (validated like 240-242); out
 * d_reward[n], d_done[n], d_reason[n] (as gc_env_step), and optionally (NULL = skip)
 * d_mask[65][n] (legal-action mask of the new position, WORD-MAJOR: word f of board i at
 * d_mask[f * n + i] = targets of from-square f, word 64 bit c = action 4096 + c -- each of
 * the kernel's mask stores then writes 512 contiguous bytes; gc_env_legal_mask's host layout
 * is the transpose),
 * d_obs[n][64] (int8 board, the observation of 153-158), d_count[n] (legal actions),
 * d_pick[n] (a uniform Philox pick over the new list, the k-th legal action in action-id
 * order -- the mask's order; also the env's next policy action).  flags bit 0: auto-reset finished boards (the mask / obs / pick then describe
 * the new episode).  Asynchronous on the env's stream: order your own work with it through
 * gc_env_get_stream (a hipStream_t) or gc_env_synchronize.  Reference rules only. */
int gc_env_step_device(gc_env* e, const uint16_t* d_actions, int32_t* d_reward, uint8_t* d_done,
                       uint8_t* d_reason, uint64_t* d_mask, int8_t* d_obs, int32_t* d_count,
                       uint16_t* d_pick, int flags);
/* gc_env_step_device with the mask's row stride in words (>= n; 0 = n, the packed form above):
 * word f of board i at d_mask[f * mask_stride + i].  With n a multiple of a large power of two,
 * packed rows (512 KiB apart at n = 65 536) fall on the same HBM channels; a padded stride
 * spreads them.  The stride is an argument of every call (no state kept on the env). */
int gc_env_step_device2(gc_env* e, const uint16_t* d_actions, int32_t* d_reward, uint8_t* d_done,
                        uint8_t* d_reason, uint64_t* d_mask, int8_t* d_obs, int32_t* d_count,
                        uint16_t* d_pick, int flags, int64_t mask_stride);
int gc_env_get_stream(gc_env* e, void** stream);
/* device memory helpers for callers without an allocator; kind 0 h2h 1 h2d 2 d2h 3 d2d
 * (synchronous on the env's stream) */
int gc_device_alloc(int device, uint64_t bytes, void** ptr);
int gc_device_free(int device, void* ptr);
int gc_env_copy(gc_env* e, void* dst, const void* src, uint64_t bytes, int kind);
/* Device-resident random self-play (the test_benchmark.py driver): n_plies one-ply kernel
 * launches; each ply = one env.step() with a uniform Philox pick over the legal list, a
 * reset when done, a reset without a step when the list is empty (reason 4).  The policy's
 * rank (agent and random opponent, both rule sets) indexes the legal moves in move-set order
 * (gc_core.h sw_gen: pawn / knight / slider-direction / king-step target sets, then castles);
 * gc_env_step_device's `pick` output indexes them in action-id order (its mask's order). */
int gc_env_step_random(gc_env* e, int n_plies);
/* gc_env_step_random over k board ranges on k streams of the device (k in [1, 8]; default
 * from GC_STREAMS, else 2): a range's ply p+1 waits only for its own ply p, so the ranges'
 * launches overlap each other's ramp and tail.  Results are independent of k. */
int gc_env_set_streams(gc_env* e, int k);
/* 1 when gc_env_step_random / gc_env_rollout (without traces) run the paired two-wave
 * kernels for this env's rules and opponent mode, 0 when the one-wave kernels run (the
 * random opponent from a start position without a pick table, or whose opening can leave
 * both kings checked), -1 on error.  Results are the same either way. */
int gc_env_paired(gc_env* e);
/* waves per 64 boards of this env's fused rollout (gc_env_rollout / gc_env_rollout_device):
 * 4 (k_env_rollout4: self-play under the reference rules, unless GC_NO_QUAD is set), 2 (the
 * paired k_env_rollout2) or 1 (the one-wave kernels); -1 on error.  Results are the same. */
int gc_env_rollout_waves(gc_env* e);
/* the fewest plies per launch of k_env_rollout4 that run with the 3-fold window's occupancy
 * filter in LDS (shorter launches probe the window's table every ply); the filter needs a
 * board's window emptied inside the launch before it applies.  Results are the same. */
int gc_env_rollout_occ_min_plies(void);
/* re-pick policy actions for the current states (after set_states / external steps) */
int gc_env_select_random(gc_env* e);
/* Same driver fused into ONE launch of n_plies plies (state kept in registers).  Optional
 * host traces of n_plies*n entries ([ply][board]); stats8 = {steps, sum(reward), ends by
 * reason 0..5} summed over boards (may be NULL). */
int gc_env_rollout(gc_env* e, int n_plies, int16_t* tr_action, int16_t* tr_reward, uint8_t* tr_done,
                   uint8_t* tr_reason, uint64_t* stats8);
/* n_plies env.step() calls of every board under the random self-play policy (the
 * test_benchmark.py:17-31 driver, opponent as configured), issued as ONE launch per 16 383
 * plies with the state held in registers, asynchronous on the env's stream (no host sync).
 * d_trace: NULL, or device memory of n_plies*n uint64 words ([ply][board]) receiving every
 * ply's outputs: bits 0-15 action played (int16, -1 = none: the driver's no-move reset),
 * 16-31 reward (int16), 32-39 done, 40-47 reason.  Afterwards the env is in the state
 * n_plies gc_env_step_random plies leave it in (outputs = the last ply's).  ev_begin /
 * ev_end: event slots (see gc_env_record_event) recorded right before / after the launches,
 * -1 = none. */
int gc_env_rollout_device(gc_env* e, int n_plies, uint64_t* d_trace, int ev_begin, int ev_end);
int gc_env_get_outputs(gc_env* e, int32_t* reward, uint8_t* done, uint8_t* reason, uint16_t* next_action,
                       uint32_t* nsteps);
int gc_env_get_states(gc_env* e, int8_t* boards, uint8_t* meta);
int gc_env_set_states(gc_env* e, const int8_t* boards, const uint8_t* meta);
/* possible_moves of every board, reference order; moves is n*cap */
int gc_env_legal_moves(gc_env* e, uint16_t* moves, int cap, int32_t* counts);
/* legal action mask per board: 64 words (from -> targets) + 1 word (bit c: action 4096+c) */
int gc_env_legal_mask(gc_env* e, uint64_t* mask, int32_t* counts);
/* The repetition spill table of a player_color BLACK env (whose games have no move cap, so a
 * 3-fold window can outgrow its per-board table; chess_v2.py:291-292): log2 of its slots (0 =
 * none), slots in use and live entries.  Synchronous; an error if an insert ever found no
 * free slot (the table grows long before that, between calls). */
int gc_env_spill_info(gc_env* e, int* bits, uint64_t* used, uint64_t* live);
/* wait for the env's stream (spin-polls up to GC_SPIN_US, default 20 ms, then blocks) */
int gc_env_synchronize(gc_env* e);
/* wait for the work of the last gc_env_rollout_device call: when it was a quad launch
 * (gc_env_rollout_waves = 4), until its completion word -- written to host-mapped memory by
 * the launch's last workgroup after every workgroup's stores -- arrives, else as
 * gc_env_synchronize.  Later work on the env's stream (an event record) may still be pending;
 * anything read through that stream stays ordered after the launch. */
int gc_env_wait_rollout(gc_env* e);
/* FEN (host-side, no GPU): placement rank 8 first (board row 0), side to move, castling ->
 * the four *_castle_is_possible flags (chess_v2.py:301-313); en passant and the half-move
 * clock are ignored (not part of the reference's rules); full-move number n -> move_count
 * n - 1 (meta8[7]).  A bare placement field means WHITE to move, no rights, move_count 0. */
int gc_fen_to_state(const char* fen, int8_t* board, uint8_t* meta);
int gc_state_to_fen(const int8_t* board, const uint8_t* meta, char* out, int cap);
/* rules 1 (FIDE): meta[7] = en-passant file + 1 (parsed / written) instead of move_count */
int gc_fen_to_state_rules(const char* fen, int8_t* board, uint8_t* meta, int rules);
int gc_state_to_fen_rules(const int8_t* board, const uint8_t* meta, char* out, int cap, int rules);
/* Rules of the env (see gc_engine_set_rules); FIDE needs opponent "none" (its fused rollout
 * keeps no per-ply traces).  Resets every board. */
int gc_env_set_rules(gc_env* e, int rules);
/* set every board from a FEN (n strings); check flags from update_state (lib.rs:1386-1393);
 * repetition windows cleared */
int gc_env_set_fens(gc_env* e, const char* const* fens);
/* Under rules=fide the env's en-passant file per board (-1 = none) travels beside
 * get_states / set_states (meta8[7] is the env's move_count there).  set: FIDE only. */
int gc_env_get_en_passant(gc_env* e, int8_t* files);
int gc_env_set_en_passant(gc_env* e, const int8_t* files);
/* Bit-exact checkpoint / resume of the whole env (replaces ChessEnvV2's state dict getter /
 * setter, chess_v2.py:301-323, PLUS what it leaves out: the 3-fold history saved_boards
 * (192, 404-407), move_count, done, the policy streams and step counters).  The blob is
 * self-describing (header, per-board slab, the live repetition-window entries; ~80 B/board
 * + 64 B per window entry).  gc_env_load needs an env of the same size, rules, opponent mode,
 * player colour, seed and initial board; a loaded env continues exactly as the saved one
 * would have.  gc_env_save: cap = buffer size, *written = the bytes needed (also on a
 * too-small buffer). */
int gc_env_checkpoint_bytes(gc_env* e, uint64_t* bytes);
int gc_env_save(gc_env* e, void* buf, uint64_t cap, uint64_t* written);
int gc_env_load(gc_env* e, const void* buf, uint64_t size);
/* HIP events on the env's stream (8 slots) for in-process kernel timing */
int gc_env_record_event(gc_env* e, int slot);
int gc_env_elapsed_ms(gc_env* e, int a, int b, float* ms);
uint64_t gc_env_device_bytes(gc_env* e);
/* sum over boards of the current 3-fold repetition-window length (traffic accounting) */
int gc_env_window_sum(gc_env* e, uint64_t* sum);

#ifdef __cplusplus
}
#endif
#endif
