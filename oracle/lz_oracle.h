/* lz_oracle.h — CPU restatement of LightZero's batched MuZero / EfficientZero ctree.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / CPU baseline —
 * never as the thing measured or shipped. The product path (lightzero_amd/) never
 * links or calls it.
 *
 * Follows, function by function (file:line relative to /root/reference):
 *   lzero/mcts/ctree/ctree_muzero/lib/cnode.cpp        (MuZero tree, "mz")
 *   lzero/mcts/ctree/ctree_efficientzero/lib/cnode.cpp (EfficientZero tree, "ez")
 *   lzero/mcts/ctree/common_lib/cminimax.cpp           (min-max stats)
 *   lzero/mcts/ctree/common_lib/utils.cpp:25           (srand(tv_usec) -> explicit seed)
 * Pinned against the tests/golden npz transcripts (transcripts of the reference build, oracle/build_ref.sh).
 */
#ifndef LZ_ORACLE_H
#define LZ_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct lzo_tree lzo_tree;

/* glibc srandom/random TYPE_3 restatement (the stream rand() returns). */
typedef struct { uint32_t ring[31]; int f, r; } lzo_glibc_rng;
void lzo_glibc_srand(lzo_glibc_rng *g, uint32_t seed);
int32_t lzo_glibc_rand(lzo_glibc_rng *g);

/* ez != 0 selects the EfficientZero value-prefix semantics. */
lzo_tree *lzo_create(int num_roots, int action_space, int max_sims, int ez);
void lzo_destroy(lzo_tree *t);
/* legal_actions: [B][A] ascending-or-any order, padded; legal_count: [B]. */
void lzo_set_legal(lzo_tree *t, const int32_t *legal_actions, const int32_t *legal_count);
void lzo_set_delta(lzo_tree *t, float value_delta_max);
/* noises may be NULL (prepare_no_noise). noises: [B][A], i-th entry matches i-th legal action. */
void lzo_prepare(lzo_tree *t, float noise_weight, const float *noises, const float *rewards,
                 const float *logits, const int32_t *to_play);
void lzo_traverse(lzo_tree *t, int pb_c_base, float pb_c_init, float discount, uint32_t seed,
                  const int32_t *virtual_to_play, int32_t *out_x, int32_t *out_y, int32_t *out_a,
                  int32_t *out_vtp, int32_t *out_len);
/* Same walk with the LZM_RNG_FAST draw stream (Philox4x32-10 per root and level). */
void lzo_traverse_fast(lzo_tree *t, int pb_c_base, float pb_c_init, float discount, uint32_t seed,
                       const int32_t *virtual_to_play, int32_t *out_x, int32_t *out_y, int32_t *out_a,
                       int32_t *out_vtp, int32_t *out_len);
void lzo_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
void lzo_backprop(lzo_tree *t, int current_latent_state_index, float discount, const float *rewards,
                  const float *values, const float *logits, const int32_t *is_reset,
                  const int32_t *to_play);
void lzo_get_distributions(const lzo_tree *t, int32_t *out /*[B][A], -1 padded*/);
void lzo_get_values(const lzo_tree *t, float *out);
int lzo_get_trajectories(const lzo_tree *t, int32_t *out /*[B][tmax], -1 padded*/, int tmax);
/* Diagnostics (tests only). lzo_get_path_actions: root i's last traverse path as actions, returns its
 * length. lzo_path_scores: the pUCT scores cselect_child computes at each level of root i's walk down
 * `actions` (n of them) in the tree as it stands — the mean-q chain as cbatch_traverse carries it from
 * parent_q = 0 — out [n + 1][A], -inf for actions not legal at the level; returns the levels written. */
int lzo_get_path_actions(const lzo_tree *t, int i, int32_t *out, int cap);
int lzo_path_scores(const lzo_tree *t, int i, int pb_c_base, float pb_c_init, float disc, int players,
                    const int32_t *actions, int n, float *out);

/* CPU baseline: tree-only search with scripted network responses, envs partitioned over
 * `threads` pthreads (each shard its own batch + RNG stream, i.e. shard-local parity).
 * Returns wall seconds for `searches` full searches of B roots x S simulations. */
double lzo_bench_tree_only(int B, int A, int S, int threads, int searches, uint32_t seed);

/* Exhaustive-check helper: number of k in [0, n) where host libm expf(bit pattern first+k)
 * differs bitwise from got[k] (pins the device glibc-expf port, lzm_numerics.h). */
long lzo_expf_mismatches(uint32_t first, int64_t n, const float *got, int threads);

#ifdef __cplusplus
}
#endif
#endif
