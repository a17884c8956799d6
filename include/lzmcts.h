/* lzmcts.h — C ABI of the MI355X-native batched MuZero / EfficientZero MCTS tree
 * (liblzmcts.so, built from lightzero_amd/csrc/lzm_kernels.hip for gfx950).
 *
 * Drop-in boundary for LightZero's ctree (reference paths relative to /root/reference):
 *   lzero/mcts/ctree/ctree_muzero/mz_tree.pyx        (Roots, MinMaxStatsList, ResultsWrapper,
 *                                                      batch_traverse, batch_backpropagate)
 *   lzero/mcts/ctree/ctree_efficientzero/ez_tree.pyx (same, + is_reset)
 *   lzero/mcts/tree_search/mcts_ctree.py:255-321     (per-simulation loop: gather, decode)
 *   lzero/policy/scaling_transform.py:97-128         (InverseScalarTransform)
 * Each entry point below names the reference interface it replaces.
 *
 * Conventions
 *  - Every pointer argument is a DEVICE pointer (HBM), unless its name ends in _host.
 *  - `stream` is a hipStream_t passed as void* (NULL = the null stream). All calls are
 *    asynchronous on that stream and capture-safe (no host sync, no allocation) except
 *    lzm_create / lzm_reserve / lzm_destroy.
 *  - Return value: LZM_OK (0) or a negative lzm_status. No C++ exception crosses the ABI.
 *  - One handle = one batch of roots (a CRoots + the CSearchResults of its last traverse).
 *    Not thread-safe; use one handle per stream.
 *  - Min-max statistics (CMinMaxStatsList) live in a caller-owned float[B*4] device buffer,
 *    initialised by lzm_minmax_init, exactly as the reference creates one per search.
 */
#ifndef LZMCTS_H
#define LZMCTS_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct lzm_handle lzm_handle;

enum lzm_status {
  LZM_OK = 0,
  LZM_ERR_ARG = -1,      /* bad argument (null pointer, size out of range) */
  LZM_ERR_HIP = -2,      /* a HIP runtime call failed */
  LZM_ERR_CAPACITY = -3, /* latent index beyond the reserved simulations: call lzm_reserve */
  LZM_ERR_STATE = -4,    /* call order violated (e.g. backprop before traverse) */
  LZM_ERR_RESIDENCY = -5, /* a launch that needs its whole grid co-resident was refused; nothing ran */
  LZM_ERR_RANGE = -6      /* split-fp16 network values left their range (non-finite, or beyond ~2^114): the
                             outputs are not f32-exact; rerun the network with LZM_CONV_F32 */
};

enum lzm_flags {
  LZM_TREE_EZ = 1,  /* EfficientZero value-prefix tree (ctree_efficientzero) instead of MuZero */
  LZM_RNG_FAST = 2  /* per-root counter-based (Philox4x32-10) tie-break stream instead of the
                       batch-serial glibc rand() stream of the reference (parity mode) */
};

/* Creates a tree for `num_roots` roots, `action_space` actions, capacity for `max_sims`
 * simulations per search (grown by lzm_reserve). Replaces Roots.__cinit__ (mz_tree.pyx:29-32)
 * / CRoots::CRoots (ctree_muzero/lib/cnode.cpp:301-317). */
int lzm_create(int num_roots, int action_space, int max_sims, int flags, lzm_handle **out);
int lzm_destroy(lzm_handle *h); /* Roots.__dealloc__ (mz_tree.pyx:53-54) */
int lzm_reserve(lzm_handle *h, int max_sims);
int lzm_num_roots(const lzm_handle *h);
int lzm_sims_capacity(const lzm_handle *h);
int lzm_action_space(const lzm_handle *h);
int lzm_flags(const lzm_handle *h);
const char *lzm_last_error(void);

/* Builds the pUCT table {log((N+base+1)/base)+init, sqrt(N)} for these constants with the host
 * libm (synchronous H2D; call outside stream capture). lzm_traverse rebuilds it on demand. */
int lzm_set_pb_c(lzm_handle *h, int pb_c_base, float pb_c_init);

/* Copies the whole tree state (nodes, root legal lists, last search paths) of `src` into `dst`
 * (same num_roots / action_space; dst capacity >= src). */
int lzm_copy_tree(lzm_handle *dst, const lzm_handle *src, void *stream);

/* MinMaxStatsList(n) + set_delta (mz_tree.pyx:5-16, common_lib/cminimax.cpp:7-66).
 * minmax: float[n*4] = {maximum, minimum, value_delta_max, 0} per root. */
int lzm_minmax_init(float *minmax, int n, float value_delta_max, void *stream);

/* Roots.prepare / prepare_no_noise (mz_tree.pyx:34-40; cnode.cpp:321-358).
 * legal_actions: int32[B*A], row i = the legal list of root i in the caller's order, padded;
 * legal_count: int32[B]; noises: float[B*A] matched to legal order, or NULL for
 * prepare_no_noise; rewards: float[B] (value_prefix for EZ); logits: float[B*A];
 * to_play: int32[B]. */
int lzm_roots_prepare(lzm_handle *h, const int32_t *legal_actions, const int32_t *legal_count,
                      const float *noises, float noise_weight, const float *rewards,
                      const float *logits, const int32_t *to_play, void *stream);

/* batch_traverse (mz_tree.pyx:95-101; cbatch_traverse cnode.cpp:755-824).
 * seed: device uint32 read by the kernel = the srand() seed of this call (parity mode) or the
 * Philox key (fast mode). Outputs int32[B]: x = latent_state_index_in_search_path,
 * y = latent_state_index_in_batch, action = last_actions, vtp = virtual_to_play_batchs,
 * len = search_lens (ResultsWrapper.get_search_len). out_action_i64 (int64[B], may be NULL)
 * is the same action list ready to feed model.recurrent_inference. */
int lzm_traverse(lzm_handle *h, int pb_c_base, float pb_c_init, float discount, float *minmax,
                 const uint32_t *seed, const int32_t *virtual_to_play, int32_t *out_x, int32_t *out_y,
                 int32_t *out_action, int64_t *out_action_i64, int32_t *out_vtp, int32_t *out_len,
                 void *stream);

/* Leaf gather: out[i, :] = latent_pool[x[i], i, :] over a pool laid out [S+1][B][row_elems]
 * (replaces the host loop mcts_ctree.py:283-289). */
int lzm_gather_latent(lzm_handle *h, const float *latent_pool, int64_t row_elems, const int32_t *x,
                      float *out, void *stream);

/* batch_backpropagate (mz_tree.pyx:74-80; cbatch_backpropagate cnode.cpp:480-500; EZ
 * ez_tree.pyx:83-93 with is_reset, ctree_efficientzero/lib/cnode.cpp:577-601). rewards are
 * value_prefixes for EZ; is_reset int32[B] (EZ only, may be NULL for MZ). */
int lzm_backprop(lzm_handle *h, int current_latent_state_index, float discount, float *minmax,
                 const float *rewards, const float *values, const float *logits, const int32_t *to_play,
                 const int32_t *is_reset, void *stream);

/* Fused decode + expand + backup for one simulation (mcts_ctree.py:300-318 in one kernel):
 * reward/value heads given as support logits [B][support_len] (categorical != 0, softmax +
 * expectation + h^-1 as InverseScalarTransform, scaling_transform.py:118-128) or as scalars
 * [B][1] (categorical == 0, h^-1 only). lstm_horizon > 0 (EZ) applies the reset rule
 * is_reset = search_len % lstm_horizon == 0 (mcts_ctree.py:810-814) and writes it to
 * out_is_reset (int32[B], may be NULL). If next_latent and pool_slot are non-NULL the new
 * latent rows [B][row_elems] are copied into pool_slot (mcts_ctree.py:305). out_decoded
 * (float[B][2] = {reward, value} after h^-1, may be NULL) exposes what the tree consumed. */
int lzm_decode_backprop(lzm_handle *h, int current_latent_state_index, float discount, float *minmax,
                        const float *reward_logits, const float *value_logits, int support_len, int categorical,
                        const float *policy_logits, const int32_t *to_play, int lstm_horizon,
                        int32_t *out_is_reset, const float *next_latent, float *pool_slot, int64_t row_elems,
                        float *out_decoded, void *stream);

/* InverseScalarTransform.__call__ (scaling_transform.py:118-128) alone: out[i] = h^-1(E_p[support]). */
int lzm_inverse_scalar_transform(const float *logits, int rows, int support_len, int categorical, float *out,
                                 void *stream);

/* Roots.get_distributions / get_values / get_trajectories (mz_tree.pyx:43-51;
 * cnode.cpp:369-417). distributions: int32[B*A] in legal order, -1 padded;
 * values: float[B]; trajectories: int32[B*tmax], -1 padded. */
int lzm_get_distributions(lzm_handle *h, int32_t *out, void *stream);
int lzm_get_values(lzm_handle *h, float *out, void *stream);
int lzm_get_trajectories(lzm_handle *h, int32_t *out, int tmax, void *stream);

/* ---- Fused whole search for the MuZeroModelMLP family (lzero/model/muzero_model_mlp.py) ----
 * One launch runs all `num_simulations` simulations of MuZeroMCTSCtree.search
 * (mcts_ctree.py:255-321) for every root: selection, leaf-latent gather, recurrent_inference
 * (dynamics + reward head + prediction heads, BatchNorm folded into the Linears), support decode
 * (InverseScalarTransform, softmax always applied: the heads are Linear logits), expansion and
 * backup. Roots must be prepared (lzm_roots_prepare) and minmax initialised (lzm_minmax_init).
 * weights: the kernel-layout buffer written by lzm_mlp_prepare (lzm_mlp_kernel_floats() floats,
 * 16-byte aligned). lzm_mlp_prepare reads the packed network: lzm_mlp_packed_floats() floats,
 * layers in the order
 *   fc_dynamics(_1)[0] (K = hidden + actions: latent rows then one-hot action rows),
 *   fc_dynamics(_1)[1], [fc_dynamics_2[0], fc_dynamics_2[1] if res_dynamics],
 *   fc_reward_head[0] (hidden -> head_hidden), fc_reward_head[1] (head_hidden -> support),
 *   fc_prediction_common[0], [1], fc_value_head[0], [1], fc_policy_head[0], [1] (-> actions);
 * each as W[K][N] (input-major, i.e. torch weight transposed) followed by bias[N]; ReLU after
 * every layer except the three head outputs; res_dynamics adds the input latent after
 * fc_dynamics_1 (muzero_model_mlp.py:427-431). latent_pool: float[S+1][B][hidden] with slot 0 =
 * root latents; slots 1..S receive the new latents. seeds: uint32[S] (traverse k uses seeds[k]).
 * rec_* (nullable, [S][B] / [S][B][2] / [S][B][actions]): per-simulation x, last action,
 * search_len, decoded {reward, value} and policy logits. */
int64_t lzm_mlp_packed_floats(int hidden, int actions, int head_hidden, int support, int res_dynamics);
/* Kernel layout: each layer's weights in the order the search kernel's lanes stream them (one
 * contiguous 1 KiB dwordx4 read per wave-instruction), K zero-padded to a multiple of 16, then its
 * bias. Asynchronous on `stream`; re-run whenever the network's parameters change. */
int64_t lzm_mlp_kernel_floats(int hidden, int actions, int head_hidden, int support, int res_dynamics);
int lzm_mlp_prepare(int hidden, int actions, int head_hidden, int support, int res_dynamics, const float *packed,
                    float *out, void *stream);
int lzm_search_mlp(lzm_handle *h, int hidden, int head_hidden, int support, int res_dynamics, const float *weights,
                   int num_simulations, int pb_c_base, float pb_c_init, float discount, float *minmax,
                   const uint32_t *seeds, const int32_t *virtual_to_play, float *latent_pool, int32_t *rec_x,
                   int32_t *rec_a, int32_t *rec_len, float *rec_decoded, float *rec_logits, void *stream);
/* Collect-step mode of the next lzm_search_mlp calls on h (sticky; host state only, so a captured
 * launch keeps the values it was launched with; pass nulls / 0 to clear). Replaces the small
 * launches around one collect-time search (lightzero_amd.collect.DeviceSearchStep,
 * muzero.py:617-690): count (device int64) non-null: the traverse seeds are
 * (base + *count * S + k) mod 10^6 (lzm_seed_sequence's rule; the `seeds` argument may be null)
 * and, if increment, *count is incremented after the search; root_dist (int32[B*A]) / root_values (float[B])
 * non-null: the search also writes lzm_get_root_outputs' outputs; fresh_minmax: every root starts
 * from fresh min-max bounds (lzm_minmax_init with value_delta_max) instead of reading `minmax`.
 * The network-resident kernel does all of it in-kernel; the weight-streaming kernel adds one
 * launch before and one after. Replaces the glue of mcts_ctree.py:245-321 + muzero.py:660-690. */
int lzm_search_set_step(lzm_handle *h, int64_t *count, int64_t base, int increment, int32_t *root_dist,
                        float *root_values, int fresh_minmax, float value_delta_max);
/* Which kernel lzm_search_mlp launches for a batch of B roots with `actions` actions and this
 * network: 1 = network-resident (search_res_kernel, lzm_search_res.h: the config-2 shape with one
 * root per workgroup), 0 = weight-streaming (search_mlp_kernel). Host-only, no GPU work. */
int lzm_search_mlp_kind(int B, int actions, int hidden, int head_hidden, int support, int res_dynamics);
/* int32[4]: {integrity errors: look-back spin timeouts and speculation mismatches (must stay 0),
 * slices resolved serially (ties that reached an expanded child, depth unknown until the draw),
 * such ties whose depth was published early (every draw outcome gives the same depth),
 * speculation mismatches (must stay 0)} accumulated over the handle's fused searches. */
int lzm_search_diagnostics(lzm_handle *h, int32_t *out, void *stream);
/* Diagnostics: uint64[n] (n <= 1024), shader-clock cycles workgroup g of the resident kernel spent
 * waiting in the parity-mode look-back, summed over launches; zeros unless LZM_PHASE_TIMING=1. */
int lzm_debug_root_wait_cycles(lzm_handle *h, uint64_t *out_host, int n, int reset);

/* Post-search integrity check (host-synchronous on `stream`): the sticky error counters of every
 * search path on the handle — {look-back spin timeouts, draw positions beyond the coefficient
 * table, serial-traverse fixed-point failures, fused-search errors, split-fp16 range errors, 0, 0, 0}
 * into out_host[8] (nullable). Returns LZM_ERR_RANGE when word 4 is non-zero (a split-fp16 network
 * value was non-finite or out of range: rerun with LZM_CONV_F32), else LZM_ERR_STATE when any is
 * non-zero (the parity-mode tie-break stream then differs from the reference's); clear != 0 resets
 * them. No reference counterpart: the reference's draws are serial on one host thread
 * (cnode.cpp:770, :590) and cannot fail this way. */
int lzm_check_errors(lzm_handle *h, int32_t *out_host, int clear, void *stream);

/* Diagnostics: traverse passes used by the last parity-mode traverse (device int32[1]). */
int lzm_last_traverse_passes(lzm_handle *h, int32_t *out, void *stream);

/* Device-side numerics helpers exposed for exhaustive checks. */
int lzm_debug_expf(const float *x, float *out, int64_t n, void *stream);
int lzm_debug_glibc_rand(uint32_t seed, int n, int32_t *out, void *stream);
/* Shader-clock cycles per phase of the fused search, summed over workgroups, when the process
 * runs with LZM_PHASE_TIMING=1 (synchronous; reset != 0 clears the counters). Phases: 0 select,
 * 1 draw offsets + look-back, 2 leaf gather, 3 dynamics, 4 reward head + decode, 5 prediction
 * trunk, 6 value head + decode, 7 policy head, 8 latent filing, 9 expand + backup, 10 stage-in,
 * 11 write-back; 16 + 4 * step + j: network schedule step `step`, j = 0 step body (FMAs, weight
 * prefetch, reduction, store, support decode), 1 barrier. out_host holds 64 counters. */
int lzm_debug_phase_cycles(lzm_handle *h, uint64_t *out_host, int reset);
int lzm_debug_philox(const uint32_t *ctr_key /*[n][6]*/, uint32_t *out /*[n][4]*/, int n, void *stream);
/* Process teardown: synchronises the device and frees the library's process-wide device buffers (the
 * decode's verdict scratch, debug tables) while the runtime is intact. Destroy live handles first; later
 * calls re-allocate what they need. lightzero_amd runs it from an atexit hook. */
int lzm_shutdown(void);
/* The wave butterflies of the search kernels (DPP / permlane xor_partner, xor_sum, xor_max) beside the
 * __shfl_xor (ds_bpermute) forms they replace, on one wave of in float[64]; out float[16][64] (rows:
 * partner D = 1..32, __shfl_xor D = 1..32, xor_sum, shfl sum, xor_max, shfl max). Tests only. */
int lzm_debug_xor(const float *in, float *out, void *stream);
/* The fused AlphaZero search's stone-mask done / winner and DPP pUCT argmax beside the reference-order scans they
 * replace (get_done_winner's cell scan; the first strict maximum): n boards int32[n][9], scores double[n][16];
 * out int32[n][6] = {done, winner (scan), done, winner (masks), argmax (DPP), argmax (scan)}. Tests only. */
int lzm_debug_az_rules(int n, const int32_t *boards, const double *scores, int32_t *out, void *stream);

/* ---- Device collect loop, CartPole-v0 (lzero/worker/muzero_collector.py
 * :399-705, zoo/classic_control/cartpole/envs/cartpole_lightzero_env.py) ----
 * State: state double[n][4], steps int32[n], obs float[n][4] (the current root observation).
 * lzm_cartpole_reset: every env to U(-0.05, 0.05)^4 (Philox stream `seed`).
 * lzm_cartpole_collect_step, one thread per env, after a search over `obs`: select the action from
 * `visits` int32[n][A] (select_action, lzero/policy/utils.py:515-539: visits^(1/temperature)
 * sampling, or argmax when `deterministic`), record obs / action / reward / root visit counts /
 * root value (and, when `pred_value` is given, the root's predicted value for priorities,
 * muzero_collector.py:200-227) into episode slot ep_count[i] % E of rec_* ([n][E][T(+1)][...],
 * GameSegment fields, game_segment.py:129-218; the host normalises the counts as
 * store_search_stats does), step the env (gymnasium CartPole equations in float64, truncation at
 * max_steps), auto-reset finished episodes (ep_len[n][E], ep_count[n]) and write the next root's
 * obs and Dirichlet(noise_alpha) noises float[n][A]. `counter` (int64, device) keys this step's
 * Philox streams and is only read: in the collect loop the search advances it (lzm_search_set_step with
 * increment) before this epilogue runs, so step n's streams use key n + 1; a caller driving the env without
 * such a search advances it itself after each step. pred_value / rec_pred: both or neither. ep_return float[n][E]
 * (nullable): each finished episode's return, the env's eval_episode_return (the reward sum, 1 per step;
 * muzero_collector.py:596-603 logs it). */
int lzm_cartpole_reset(int n, double *state, int32_t *steps, float *obs, uint32_t seed, void *stream);
int lzm_cartpole_collect_step(int n, int A, int T, int E, const int32_t *visits, const float *root_value,
                              const float *pred_value, double *state, int32_t *steps, float *obs, float *noises,
                              float noise_alpha, float temperature, int deterministic, float *rec_obs,
                              int32_t *rec_action, float *rec_reward, int32_t *rec_visits, float *rec_value,
                              float *rec_pred, int32_t *ep_len, int32_t *ep_count, float *ep_return, int max_steps,
                              uint32_t seed, const int64_t *counter, void *stream);

/* The Atari image configs' collect step (BASELINE.json config 5; muzero_collector.py:399-705 with
 * zoo/atari/envs/atari_lightzero_env.py): one workgroup per env right after the search — select_action
 * from the root visit counts (policy/utils.py:515-539), record o_t (u8 64x64 frame), a_t, r_t, the
 * visit counts, root value (and predicted value) into the running episode slot
 * (ep_count[i] % E of rec_* [n][E][T(+1)]...), step the game, append o_{t+1} to the model's float
 * observation stack obs [n][4][64][64] (frame / 255, frame_stack_num = 4: game_segment.py:95-127),
 * auto-reset finished episodes (their final frame goes to slot row L; ep_len / ep_count advance) and
 * draw the next root's Dirichlet(noise_alpha) noise. The game is a stand-in with Breakout's action set
 * and frame format (ALE is not installed; csrc/lzm_atari.h). state int32 [n][16], cur u8 [n][4096]
 * (the newest frame), counter: the device env-step counter, read as lzm_cartpole_collect_step reads it (the
 * collect-step search has already advanced it). ep_return float[n][E] (nullable): each finished episode's
 * UNCLIPPED score (eval_episode_return, muzero_collector.py:596-603; the recorded rewards are clipped).
 * lzm_pong_reset / lzm_pong_collect_step: the same step for config 3's Pong EfficientZero with a Pong stand-in
 * (6 actions {NOOP, FIRE, RIGHT = up, LEFT = down, RIGHTFIRE, LEFTFIRE}, the agent's paddle on the right, a
 * scripted opponent, +1 / -1 per point, 21 points end the episode; ep_return: the point difference). */
int lzm_atari_reset(int n, int32_t *state, int32_t *steps, uint8_t *cur, float *obs, uint32_t seed, void *stream);
int lzm_atari_collect_step(int n, int A, int T, int E, const int32_t *visits, const float *root_value,
                           const float *pred_value, int32_t *state, int32_t *steps, uint8_t *cur, float *obs,
                           float *noises, float noise_alpha, float temperature, int deterministic, uint8_t *rec_frames,
                           int32_t *rec_action, float *rec_reward, int32_t *rec_visits, float *rec_value,
                           float *rec_pred, int32_t *ep_len, int32_t *ep_count, float *ep_return, int max_steps,
                           uint32_t seed, const int64_t *counter, void *stream);
int lzm_pong_reset(int n, int32_t *state, int32_t *steps, uint8_t *cur, float *obs, uint32_t seed, void *stream);
int lzm_pong_collect_step(int n, int A, int T, int E, const int32_t *visits, const float *root_value,
                          const float *pred_value, int32_t *state, int32_t *steps, uint8_t *cur, float *obs,
                          float *noises, float noise_alpha, float temperature, int deterministic, uint8_t *rec_frames,
                          int32_t *rec_action, float *rec_reward, int32_t *rec_visits, float *rec_value,
                          float *rec_pred, int32_t *ep_len, int32_t *ep_count, float *ep_return, int max_steps,
                          uint32_t seed, const int64_t *counter, void *stream);

/* Device packing of a collector's finished episodes for the trajectory return (SURVEY.md §8(e);
 * replaces the host loop over envs that builds GameSegments' arrays, muzero_collector.py:612-632, and
 * feeds the rank all-gather that replaces muzero_collector.py:709-712's DDP path). Episode k of env i
 * lives in slot k % E; consumed[i] counts the episodes already returned. lzm_episodes_scan (one
 * workgroup): env_ep_off [n] / env_row_off [n] exclusive prefix sums of the new episodes and their rows
 * (L + 1 each), totals int64[3] = {episodes, rows, slot overflow (a new count >= E: a returned slot
 * was overwritten)}. lzm_episodes_pack (one workgroup per env, after the host sized the outputs from
 * totals): out_index [episodes][3] = (env, L, first row), out_frames [rows][frame_bytes] (o_0..o_L of
 * each episode, copied from rec_frames [n][E][T+1][frame_bytes]), out_scalars [rows][3 + A (+1)] =
 * [action | reward | visit counts (A) | root value (| predicted value)] with each episode's row L
 * zero but for its reward column, which holds ep_return [n][E] of the slot (nullable: 0); then
 * consumed[i] = ep_count[i]. Env-major order, each env's episodes in finishing order. */
int lzm_episodes_scan(int n, int E, const int32_t *ep_count, const int32_t *consumed, const int32_t *ep_len,
                      int32_t *env_ep_off, int64_t *env_row_off, int64_t *totals, void *stream);
int lzm_episodes_pack(int n, int E, int T, int A, int has_pred, int64_t frame_bytes, const int32_t *ep_count,
                      const int32_t *ep_len, int32_t *consumed, const int32_t *env_ep_off, const int64_t *env_row_off,
                      const void *rec_frames, const int32_t *rec_action, const float *rec_reward,
                      const int32_t *rec_visits, const float *rec_value, const float *rec_pred,
                      const float *ep_return, void *out_frames, float *out_scalars, int64_t *out_index,
                      void *stream);

/* The representation network's DownSample stages (lzero/model/common.py:164-265: conv 3x3/2 -> 32, a 32-channel
 * residual block at 32 x 32, the downsample block (3x3/2 -> 64 with a 3x3/2 shortcut), a 64-channel residual
 * block at 16 x 16, avg_pool 3x3/2) of the conv MuZeroModel / EfficientZeroModel, BatchNorm folded, on the
 * split-fp16 matrix path (two fp16 terms per f32 operand, three MFMA products per K; csrc/lzm_repr.h): 7
 * convolution launches with fused bias / residual / ReLU and a pool launch. lzm_repr_prepare packs raw =
 * [conv1 W (32 x cin x 9), b (32) | block1 W1 (32 x 32 x 9), b1, W2, b2 |
 * down W1 (64 x 32 x 9), b1 (64), W2 (64 x 64 x 9), b2 (64), W3 (64 x 32 x 9) | block2 W1 (64 x 64 x 9), b1, W2,
 * b2] into lzm_repr_floats() floats (every weight row scaled by a power of two, its inverse kept for the
 * epilogue; each tile's input split after scaling by a power of two from its exact max: lzm_conv.h's range
 * rule). lzm_repr_downsample: obs f32 NCHW [B][cin][64][64] -> out [B][64][8][8] (the input of
 * lzm_conv_resnet8_p's 8 x 8 tail); ws: lzm_repr_workspace_floats(B) floats (NHWC stages). */
int64_t lzm_repr_floats(void);
int lzm_repr_prepare(int cin, const float *raw, float *out);
int64_t lzm_repr_workspace_floats(int B);
int lzm_repr_downsample(int B, int cin, const float *weights, const float *obs, float *ws, float *out, void *stream);

/* The BatchNorm-folded conv representation network's epilogue in one pass (conv_infer.FoldedConvInitial,
 * replacing torch's bias broadcast add, residual add and ReLU passes after each MIOpen convolution,
 * lzero/model/common.py:164-265): y[n][c][p] = max((y[n][c][p] + bias[c]) + z[n][c][p], 0) in place,
 * z nullable (no residual), relu 0 keeps the sum. y, z contiguous [N][C][HW], HW % 4 == 0, 16-B
 * aligned. The same float additions in the same order as the torch passes (the same bits). */
int lzm_bias_add_relu(float *y, const float *bias, const float *z, int N, int C, int HW, int relu, void *stream);

/* ---- batched AlphaZero for TicTacToe (replaces MCTS.get_next_action,
 * lzero/mcts/ctree/ctree_alphazero/mcts_alphazero.cpp:131-207, called per env from
 * lzero/policy/alphazero.py:266 and :327). B boards are searched together on the device; the caller
 * evaluates the network between launches. Per search:
 *   lzm_az_begin            boards int32[B][9] (0/1/2), start_player_index int32[B] -> state float[B][27]
 *                           (current_state / 2 of every root, the network input)
 *   network(state)          -> probs float[B][pstride >= 9] (softmax over the 9 actions), values float[B]
 *   lzm_az_step(sim = -1)   expand the roots (+ default-seeded Dirichlet noise when with_noise), descend
 *                           for simulation 0, write its leaf states
 *   for sim in 0..S-1: network(state); lzm_az_step(sim)   finish simulation `sim`, descend for sim + 1
 *   lzm_az_finish           visits int32[B][9], probs double[B][9] (visit_count_to_action_distribution),
 *                           action int32[B] (first argmax, or a Philox draw keyed by seed, *counter, board)
 * `ws` is a device buffer of lzm_az_workspace_bytes(B, S); lzm_az_set_constants fills its pUCT tables
 * (glibc log / sqrt over the integer parent count) and noise table once (synchronous). The state
 * buffer is overwritten by every begin / step. Everything but set_constants is graph-capturable. */
int lzm_az_workspace_bytes(int B, int S, int64_t *out);
int lzm_az_noise_table(double alpha, int max_n, double *out_host); /* host: row n-1 = vector for n children */
int lzm_az_set_constants(int B, int S, void *ws, double pb_c_base, double pb_c_init, double alpha, void *stream);
int lzm_az_begin(int B, int S, void *ws, const int32_t *boards, const int32_t *start_index, float *state,
                 void *stream);
int lzm_az_step(int B, int S, void *ws, int sim, const float *probs, int pstride, const float *values, int vstride,
                int with_noise, double noise_weight, float *state, void *stream);
int lzm_az_finish(int B, int S, void *ws, double temperature, int sample, uint32_t seed, const int64_t *counter,
                  int32_t *visits, double *probs, int32_t *action, void *stream);
/* test access: node visit / value_sum / first-child rows [B][1 + 9 (S + 1)] and node counts [B] (any may be NULL) */
int lzm_az_export_tree(int B, int S, void *ws, int32_t *visit, float *vsum, int32_t *first, int32_t *nnodes,
                       void *stream);

/* ---- fused AlphaZero search: the TicTacToe config's AlphaZeroModel (alphazero_model.py:14-330; 16 channels,
 * num_res_blocks 1 or 2, head width 8, 9 actions, scalar value) evaluated inside the search kernel; one
 * launch per search of B boards (tree in LDS). Same inputs / outputs / ws / constants as lzm_az_begin ..
 * lzm_az_finish; export_tree != 0 also writes the final trees into ws (lzm_az_export_tree).
 * Weights: lzm_az_net_prepare(nres, raw, out) packs, on the host, `raw` =
 *   conv0 W[16][27] (out, in*9 + tap), b[16];  4*nres x { conv W[16][144], b[16] } (representation
 *   blocks' conv1, conv2, then the prediction's; BatchNorm folded in);  1x1 W[32][16] (value rows, then
 *   policy rows), b[32];  head block [2448]: value FC1 [8][144] @0, b @1152, LN gamma @1160, beta @1168,
 *   FC2 [8] @1176, b @1184; policy FC1 [8][144] @1188, b @2340, gamma @2348, beta @2356, FC2 [9][8]
 *   @2364, b [9] @2436
 * into lzm_az_net_floats(nres) floats, to be copied to the device.
 * lzm_az_net_eval: the same network on state float[n][27] -> probs float[n][9], value float[n]
 * (bit-identical to what the fused search computes for that input). */
int64_t lzm_az_net_floats(int nres);
int lzm_az_net_prepare(int nres, const float *raw, float *out_host);
int lzm_az_net_eval(int nres, const float *weights, const float *state, int n, float *probs, float *value,
                    void *stream);
int lzm_az_search_fused(int B, int S, void *ws, int nres, const float *weights, const int32_t *boards,
                        const int32_t *start_index, int with_noise, double noise_weight, double temperature,
                        int sample, uint32_t seed, const int64_t *counter, int32_t *visits, double *probs,
                        int32_t *action, int export_tree, void *stream);

/* ---- convolutional recurrent trunk (configs 3 / 5: conv MuZeroModel / EfficientZeroModel) --------
 * The conv part of recurrent_inference (muzero_model.py:505-530, efficientzero_model.py:526-574,
 * common.py:854-881) with eval BatchNorm folded, one workgroup per env (lzm_conv.h): dynamics conv over
 * the gathered latent + action map + residual, n_dres basic blocks -> next latent; 1x1 reward conv;
 * n_pres basic blocks; stacked 1x1 value/policy head conv. Latent 64 x 8 x 8 only.
 * lzm_conv_trunk_prepare packs, on the host, raw = dyn W[64][64][9] (latent input channels);
 *   n_dres x { W1[64][64][9], b1[64], W2[64][64][9], b2[64] };  reward W[r_ch][64], b[r_ch];
 *   n_pres x { same };  head W[h_ch][64], b[h_ch]
 * into lzm_conv_trunk_floats() floats (copy to the device, 16-byte aligned). The split layout also holds each
 * layer's weight-row scales and the bounds its activation scales are derived from (lzm_conv.h, "Range");
 * the dynamics conv's bias bound is max |actmap|: set it with lzm_conv_trunk_actmap_bound before the copy.
 * lzm_conv_trunk: input latent of env b = pool[(x[b] * B + b) * 4096 ..] (x nullable: pool[b * 4096]);
 * actmap float[A][64][64] (action planes' conv + dynamics bias), action int32[B];
 * outputs out_latent float[B][4096], out_r float[B][r_ch*64], out_h float[B][h_ch*64].
 * The unsuffixed entry points run the exact-f32 matrix path (LZM_CONV_F32); the _p forms take the
 * precision: LZM_CONV_F32 (v_mfma_f32_32x32x2_f32) or LZM_CONV_SPLIT (each f32 operand split into two
 * fp16 terms, three products per K on v_mfma_f32_16x16x32_f16, every weight row and activation tensor scaled
 * by a power of two so both terms stay normal fp16: f32-level error, 2^-22 per operand; the EfficientZero
 * LSTM gate GEMM on the same split). err (nullable, device int32): counts envs whose split activations were
 * non-finite or beyond the scales' range (lzm_error_word(h, 4) reports them through lzm_check_errors). A blob
 * packed for one precision must be run with the same precision. LZM_CONV_BF16X3 is the split precision's
 * former name. */
#define LZM_CONV_F32 0
#define LZM_CONV_SPLIT 1
#define LZM_CONV_BF16X3 LZM_CONV_SPLIT
int64_t lzm_conv_trunk_floats(int n_dres, int n_pres);
int lzm_conv_trunk_prepare(int n_dres, int n_pres, int r_ch, int h_ch, const float *raw, float *out_host);
int lzm_conv_trunk(int B, int n_dres, int n_pres, int r_ch, int h_ch, const float *weights, const float *actmap,
                   const float *pool, const int32_t *x, const int32_t *action, float *out_latent, float *out_r,
                   float *out_h, void *stream);
int64_t lzm_conv_trunk_floats_p(int n_dres, int n_pres, int precision);
int lzm_conv_trunk_prepare_p(int precision, int n_dres, int n_pres, int r_ch, int h_ch, const float *raw,
                             float *out_host);
int lzm_conv_trunk_actmap_bound(int n_dres, int n_pres, float actmap_absmax, float *packed_host);
int lzm_conv_trunk_p(int precision, int B, int n_dres, int n_pres, int r_ch, int h_ch, const float *weights,
                     const float *actmap, const float *pool, const int32_t *x, const int32_t *action,
                     float *out_latent, float *out_r, float *out_h, int32_t *err, void *stream);
/* The conv representation network's 8 x 8 tail on the same split-bf16 trunk kernel (no dynamics conv,
 * no reward 1x1): in [B][64][8][8] (the DownSample's output after its last average pool) through
 * n_blocks residual blocks -> out_latent [B][64 * 64] (the initial latent), then n_pres prediction
 * blocks and the head 1x1 (+ ReLU) -> out_h [B][h_ch * 64]. Replaces those layers of
 * conv_infer.FoldedConvInitial (lzero/model/common.py:369-465 representation blocks, :568-640
 * prediction trunk). Weights: lzm_conv_trunk_prepare_p(LZM_CONV_BF16X3, n_blocks, n_pres, 1, h_ch, raw)
 * with a zero dynamics conv and a zero 1-channel reward 1x1 in raw. */
int lzm_conv_resnet8_p(int B, int n_blocks, int n_pres, int h_ch, const float *weights, const float *in,
                       float *out_latent, float *out_h, int32_t *err, void *stream);
/* lzm_conv_trunk_p writing the EfficientZero LSTM input row directly (mcts_ctree.py:776-790 +
 * efficientzero_model.py:551-556: nn.LSTM over [reward planes | leaf hidden state]): row b of xin
 * (xin_stride floats, >= r_ch*64 + H) gets the reward planes at [0, r_ch*64) and, when hpool
 * (float[.][B][H], H % 4 == 0) is given, the leaf's hidden state hpool[x[b]][b] at [r_ch*64, +H)
 * — the gather + concat that lzm_ez_lstm_input would do as a separate launch — and (split precision) xscale[b]
 * (int32 [B], required with hpool) the row's split scale exponent 14 - floor(log2 max(max reward plane, 1)) that
 * lzm_ez_lstm_step reads. */
int lzm_conv_trunk_xin_p(int precision, int B, int n_dres, int n_pres, int r_ch, int h_ch, const float *weights,
                         const float *actmap, const float *pool, const int32_t *x, const int32_t *action,
                         float *out_latent, float *xin, int xin_stride, const float *hpool, int H, int32_t *xscale,
                         float *out_h, int32_t *err, void *stream);

/* The MLP heads of the conv recurrent step in one launch (lzm_heads.h): reward hidden from
 * r [B][Kr] (optionally relu(r * r_scale + r_shift), the EfficientZero value-prefix BatchNorm),
 * value / policy hiddens from the head planes hd [B][Khd] (value planes at 0, policy planes at
 * off_policy), then the three output layers. Replaces, per simulation, the fc_reward_head /
 * fc_value / fc_policy MLPs of muzero_model.py:505-530, efficientzero_model.py:526-574 and
 * common.py:854-881 (BatchNorm folded). w1t float[3][8][32][32][4], b1[96], w2t float[32][Vr+Vv+A],
 * b2[Vr+Vv+A] as packed by lightzero_amd.conv_infer; outputs reward [B][Vr], value [B][Vv],
 * policy [B][A]. norm_words (nullable, int32 [2 * ceil(B / 2)]): also write ensure_softmax's
 * verdict for the reward and value rows (scaling_transform.py:36-62) in the layout
 * lzm_decode_backprop reads after lzm_set_norm_words, so it launches no check of its own. r = NULL: the
 * prediction heads only (value, policy; initial_inference's prediction network, common.py:854-881): Kr,
 * r_scale / r_shift, reward and norm_words are not read. */
int lzm_conv_heads(int B, int Kr, int Khd, int off_policy, const float *r, const float *r_scale, const float *r_shift,
                   const float *hd, const float *w1t, const float *b1, const float *w2t, const float *b2, int Vr,
                   int Vv, int A, float *reward, float *value, float *policy, int32_t *norm_words, void *stream);
/* lzm_conv_heads' prediction heads (r = NULL form) followed, in the same launch, by lzm_roots_prepare on `h`
 * (B roots, A <= 256 actions) with the policy logits just computed — the conv policies' initial_inference +
 * roots.prepare (muzero.py:643-660, efficientzero.py:555-575) without the preparation launch; the same root
 * records bit for bit (the policy-head workgroups prepare their envs from their LDS copy of the logits). */
int lzm_conv_heads_prepare(lzm_handle *h, int B, int Khd, int off_policy, const float *hd, const float *w1t,
                           const float *b1, const float *w2t, const float *b2, int Vr, int Vv, int A, float *value,
                           float *policy, const int32_t *legal, const int32_t *count, const float *noises,
                           float noise_weight, const float *rewards, const int32_t *to_play, void *stream);

/* One launch = one whole MuZeroMCTSCtree.search for the conv MuZeroModel (Atari configs; replaces
 * the per-simulation loop of mcts_ctree.py:255-321 around muzero_model.py:241-373's recurrent step:
 * batch_traverse, recurrent_inference, InverseScalarTransform, batch_backpropagate). Workgroup b
 * runs every simulation of root b with its tree slice in LDS: the walk (parity mode: draw-free,
 * depth flag, look-back over earlier roots only when a draw value is needed), the split-bf16 MFMA
 * trunk from latent_pool[x][b] (next latent filed into latent_pool[k + 1][b]), the head MLPs, the
 * support decode, expand and backup — the generic path's arithmetic, so the same results bit for
 * bit. Weights: trunk_w / actmap from lzm_conv_trunk_prepare_p(precision 1) and the fold's action
 * map; w1t / b1 / b2 in lzm_conv_heads' layouts, w2q its output layer as float4s [8][Vr + Vv + A][4] (k = 4 k4 .. 4 k4 + 3). latent_pool [S + 1][B][64 * 64] (slot 0 =
 * root latents), minmax float4 [B] (fresh bounds), seeds uint32 [S] (the srand(tv_usec) values),
 * rec_* (nullable): per-simulation x / action / search_len int32 [S][B], decoded {reward, value}
 * float [S][B][2], policy logits float [S][B][A]. Requires B <= the device's CU count (the grid is
 * co-resident). Errors of the tie-break stream and undecidable ensure_softmax verdicts are
 * reported by lzm_check_errors. */
int lzm_search_conv(lzm_handle *h, int num_simulations, int pb_c_base, float pb_c_init, float discount, float *minmax,
                    const uint32_t *seeds, const int32_t *vtp_in, float *latent_pool, const float *trunk_w,
                    const float *actmap, int n_dres, int n_pres, int r_ch, int h_ch, const float *w1t,
                    const float *b1, const float *w2q, const float *b2, int Kr, int Khd, int off_policy, int Vr,
                    int Vv, int categorical, int32_t *rec_x, int32_t *rec_a, int32_t *rec_len, float *rec_decoded,
                    float *rec_logits, void *stream);

/* The whole EfficientZeroMCTSCtree.search (mcts_ctree.py:696-827) for the conv EfficientZeroModel in ONE
 * launch (EZ trees): lzm_search_conv's per-root flow with the value-prefix tree (ctree_efficientzero
 * cnode.cpp:173-212, :482-575, :756-814) plus the reward LSTM step (efficientzero_model.py:526-574) as
 * lzm_ez_lstm_step's split-K tiles spread over the same grid: each root publishes its LSTM input row
 * [reward planes | hpool[x][b]] with its search_len, the tiles run the gate GEMM + cell for 64 rows x 16
 * units and hand the h1 rows back; c state filed into cpool[k + 1] and h state into hpool[k + 1],
 * zeroed where search_len % horizon == 0 (mcts_ctree.py:810-813). hpool / cpool [S + 1][B][H] (slot 0
 * = the roots' reward_hidden_state), lstm_frag = lzm_ez_lstm_prepare(W [4H][r_ch * 64 + H]),
 * lstm_bias [4H] = b_ih + b_hh, vp_s / vp_t the value-prefix BatchNorm as an affine map; heads as
 * lzm_search_conv with the reward head reading relu(h1 * vp_s + vp_t) (K = H). rec_reset (nullable)
 * is_reset int32 [S][B]. Same results as the generic path (traverse, lzm_conv_trunk_xin_p,
 * lzm_ez_lstm_step, lzm_conv_heads, lzm_decode_backprop) bit for bit. Requires max(B, 2 T) <= the
 * device's CU count, T = ceil(B / 64) * H / 16: the grid must be co-resident. When the static bound
 * (occupancy per CU x CUs; LZM_RESIDENCY_CUS=<n> caps the CU count, for tests) cannot hold it the call
 * returns LZM_ERR_RESIDENCY without running anything and the caller takes the generic path; otherwise it
 * is a plain launch (eager or captured), whose bounded hand-off waits count a timeout in the tree's
 * error word when other work on the GPU keeps part of the grid from running. */
int lzm_search_conv_ez(lzm_handle *h, int num_simulations, int pb_c_base, float pb_c_init, float discount,
                       float *minmax, const uint32_t *seeds, const int32_t *vtp_in, float *latent_pool, float *hpool,
                       float *cpool, int H, int horizon, const float *trunk_w, const float *actmap, int n_dres,
                       int n_pres, int r_ch, int h_ch, const float *lstm_frag, const float *lstm_bias,
                       const float *vp_s, const float *vp_t, const float *w1t, const float *b1, const float *w2q,
                       const float *b2, int Khd, int off_policy, int Vr, int Vv, int categorical, int32_t *rec_x,
                       int32_t *rec_a, int32_t *rec_len, float *rec_decoded, float *rec_logits, int32_t *rec_reset,
                       void *stream);

/* lzm_decode_backprop of simulation `cur` fused with lzm_traverse of the next simulation (parity /
 * glibc mode only): one launch in which the wave that backs up root i then walks root i again
 * (same requests, draws and outputs as the two separate calls). Replaces the pair
 * batch_backpropagate(sim) + batch_traverse(sim + 1) of mcts_ctree.py:255-321 / :756-827
 * (cnode.cpp:480-500, :755-824). Arguments: those of lzm_decode_backprop, then those of lzm_traverse
 * (the next traverse's seed; its outputs overwrite the current request buffers). */
int lzm_decode_backprop_traverse(lzm_handle *h, int current_latent_state_index, float discount, float *minmax,
                                 const float *reward_logits, const float *value_logits, int support_len,
                                 int categorical, const float *policy_logits, const int32_t *to_play,
                                 int lstm_horizon, int32_t *out_is_reset, const float *next_latent, float *pool_slot,
                                 int64_t row_elems, float *out_decoded, int pb_c_base, float pb_c_init,
                                 const uint32_t *seed, const int32_t *virtual_to_play_in, int32_t *out_x,
                                 int32_t *out_y, int32_t *out_last_action, int64_t *out_last_action_i64,
                                 int32_t *out_virtual_to_play, int32_t *out_search_len, void *stream);

/* lzm_get_distributions and lzm_get_values in one launch (get_distributions / get_values,
 * cnode.cpp:369-417): dist int32 [B][A] (legal order, -1 padded), values float [B]. */
int lzm_get_root_outputs(lzm_handle *h, int32_t *dist, float *values, void *stream);

/* The S traverse seeds of one collect step, usec_k = (base + count * S + k) mod 10^6 with the step
 * counter read on the device (int64 [1]); the deterministic stand-in for the reference's per-call
 * srand(tv_usec) (common_lib/utils.cpp:25) used by lightzero_amd.collect.DeviceSearchStep. */
int lzm_seed_sequence(const int64_t *count, int64_t base, int S, int32_t *seeds, void *stream);

/* Verdict words for the following lzm_decode_backprop(_traverse) calls on this handle: written by
 * lzm_conv_heads(norm_words) for the same outputs; null restores the decode's own check launch. */
int lzm_set_norm_words(lzm_handle *h, const int32_t *words);

/* ReZero search-with-reuse inputs for the following lzm_traverse / lzm_backprop /
 * lzm_decode_backprop(_traverse) calls on this handle (device arrays [B], kept by pointer; null /
 * null turns it off). With them set the traverse scores the root's true_action child by
 * carm_score and ends the walk there (x = -1 when that child is already expanded), and the backup
 * skips the expansion of such roots and backs up reuse_value for them and for roots that stopped
 * at the unexpanded true-action child. Replaces batch_traverse_with_reuse /
 * batch_backpropagate_with_reuse (mz_tree.pyx:84-107; ctree_muzero/lib/cnode.cpp:502-546,
 * 598-642, 702-749, 827-927). MuZero trees, parity mode, look-back traverse only. */
int lzm_set_reuse(lzm_handle *h, const int32_t *true_action, const float *reuse_value);

/* MuZeroModelMLP.initial_inference in one launch (lzm_initial.h): representation (Linear O->H + BN,
 * GELU(tanh), Linear H->H, SimNorm over groups of `group`) and prediction (two Linear H->H + BN +
 * ReLU; value head Linear H->F + BN + ReLU, Linear F->V; policy head Linear H->F + BN + ReLU,
 * Linear F->A) for B observations [B][O]. Replaces model.initial_inference in the collect step
 * (muzero.py:617-690; muzero_model_mlp.py:145-177, common.py:467-517, :883-971). `weights` (device)
 * holds eight BN-folded layers W[K][N] + bias[N]; `offsets` (host, 16 entries) their float offsets
 * in the order R1 w, R1 b, R2 w, R2 b, P1, P2, V1, V2, Q1, Q2. Outputs latent [B][H], value logits
 * [B][V], policy logits [B][A]. */
int lzm_mlp_initial_inference(int B, int O, int H, int F, int V, int A, int group, const float *obs,
                              const float *weights, const int64_t *offsets, float *latent, float *value, float *policy,
                              void *stream);
/* lzm_mlp_initial_inference followed, in the same launch, by lzm_roots_prepare on `h` (B roots, A
 * actions) with the policy logits just computed — MuZeroPolicy._forward_collect's initial_inference +
 * roots.prepare (muzero.py:643-660) without a second launch; the same root records bit for bit. */
int lzm_mlp_initial_inference_prepare(lzm_handle *h, int B, int O, int H, int F, int V, int A, int group,
                                      const float *obs, const float *weights, const int64_t *offsets, float *latent,
                                      float *value, float *policy, const int32_t *legal, const int32_t *count,
                                      const float *noises, float noise_weight, const float *rewards,
                                      const int32_t *to_play, void *stream);

/* EfficientZero reward LSTM, input side (lzm_lstm.h): xin[b] = [r[b] | hpool[x[b]][b]] — the leaf's
 * hidden-state gather and the concat ahead of the gate GEMM. Replaces the per-simulation gathers of
 * the LSTM state lists (mcts_ctree.py:756-775) and the nn.LSTM input assembly
 * (efficientzero_model.py:526-574). r [B][Kr], hpool [slots][B][H], xin [B][Kr + H]; Kr, H % 4 == 0. */
int lzm_ez_lstm_input(int B, int Kr, int H, const float *r, const float *hpool, const int32_t *x, float *xin,
                      void *stream);

/* EfficientZero reward LSTM, cell side: gates [B][4H] (= xin W^T + b, nn.LSTM order i, f, g, o),
 * c0 = cpool[x[b]][b]; writes h1 / c1 [B][H] and the next state slot hslot / cslot [B][H], zeroed
 * where search_len[b] % horizon == 0 (mcts_ctree.py:810-813). */
int lzm_ez_lstm_cell(int B, int H, const float *gates, const float *cpool, const int32_t *x, const int32_t *search_len,
                     int horizon, float *h1, float *c1, float *hslot, float *cslot, void *stream);

/* EfficientZero reward LSTM in one launch: the gate GEMM gates = xin W^T + bias on split-bf16 MFMA
 * with the cell (lzm_ez_lstm_cell's operations) in its epilogue — replaces the nn.LSTM step
 * (efficientzero_model.py:526-574) and the state bookkeeping of mcts_ctree.py:756-816 that the
 * rocBLAS GEMM + lzm_ez_lstm_cell pair did in two launches. xin [B][K] (K = Kr + H, % 64 == 0),
 * wfrag = lzm_ez_lstm_prepare(W [4H][K], nn.LSTM gate order i, f, g, o), bias [4H], c0 =
 * cpool[x[b]][b]; writes h1 / c1 [B][H] and the next state slot hslot / cslot (zeroed where
 * search_len[b] % horizon == 0). H % 16 == 0. Within f32 tolerance of the f32 GEMM (rtol 1e-4): each gate
 * column's weights packed scaled by a power of two (the inverse scales follow the fragments), each row's
 * 64-K stage split after scaling by a power of two from its exact max. */
int64_t lzm_ez_lstm_frag_floats(int K, int H);
int lzm_ez_lstm_prepare(int K, int H, const float *W, float *out);
/* workspace (optional, zero-filled once): lzm_ez_lstm_workspace_bytes(B, H) bytes; with it the K range
 * is split over two workgroups per tile when every workgroup fits on the GPU at once (err: a sticky
 * int32 counting hand-off timeouts, required with the workspace). */
int64_t lzm_ez_lstm_workspace_bytes(int B, int H);
/* test support: n workgroups, each holding a CU (its whole LDS) for usec microseconds, on `stream` — another
 * stream's kernel occupying CUs while a co-resident grid (lzm_search_conv_ez) launches */
int lzm_debug_hold_cus(int n, int usec, void *stream);
/* diagnostics: lzm_ez_lstm_step launches record shader-clock stamps into buf [blocks][8] (nullptr: off) */
int lzm_debug_lstm_stamps(void *buf);
/* diagnostics: lzm_az_search_fused launches add their per-phase shader-clock cycles into the device uint64[8]
 * buf ({descend, convolutions, 1x1 heads, 0, FC1/LayerNorm/FC2/softmax, expand+backup, kernel, simulations}
 * summed over workgroups; nullptr: the production instantiation) */
int lzm_debug_az_stamps(void *buf);
/* Device address of the handle's sticky error word i (0..7) for kernels launched outside the handle
 * (word 3: lzm_ez_lstm_step's hand-off timeouts, word 4: split-fp16 range errors, word 5: the one-launch conv
 * searches' abort word — set by their first wait that times out (200 ms), after which every wait of that launch
 * returns at once); lzm_check_errors reports them (and clears word 5 with the rest). */
int32_t *lzm_error_word(lzm_handle *h, int i);
/* xscale [B]: each row's split scale exponent (lzm_conv_trunk_xin_p writes it; any s with |x 2^s| < 2^15 over the
 * row is correct, 14 - floor(log2 max |row|) keeps the most bits); range_err (nullable): counts split values
 * out of fp16's range (lzm_error_word(h, 4)). */
int lzm_ez_lstm_step(int B, int K, int H, const float *xin, const int32_t *xscale, const float *wfrag,
                     const float *bias, const float *cpool, const int32_t *x, const int32_t *search_len, int horizon,
                     float *h1, float *c1, float *hslot, float *cslot, void *workspace, int32_t *err,
                     int32_t *range_err, void *stream);

#ifdef __cplusplus
}
#endif
#endif
