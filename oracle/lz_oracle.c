/* lz_oracle.c — CPU restatement of LightZero's batched MuZero / EfficientZero ctree.
 *
 * TEST INFRASTRUCTURE ONLY (see lz_oracle.h). Compiled with -O2 -ffp-contract=off so that
 * every float expression rounds exactly like the reference's SSE build (no FMA).
 * expf / logf / sqrtf are the host libm functions the reference calls (SURVEY.md §7 hard
 * part 2); rand() is restated (glibc TYPE_3) so the stream is explicit and checkable.
 *
 * Tree layout: per root, a flat node pool. The node expanded with latent index L (root: 0,
 * the leaf of simulation k: k+1) owns children slots [1 + A*L, 1 + A*L + A). That is the
 * same information the reference keeps in std::map<int, CNode> children
 * (ctree_muzero/lib/cnode.h:26), addressed without allocation.
 */
#include "lz_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define LZO_FLOAT_MAX 1000000.0f /* common_lib/cminimax.h:9 */
#define LZO_FLOAT_MIN (-LZO_FLOAT_MAX)

/* ---------------------------------------------------------------- glibc rand restatement */
/* glibc __srandom_r / __random_r, TYPE_3 (degree 31, separation 3): state[i] =
 * 16807*state[i-1] mod (2^31-1) by Schrage's method, front pointer at state[3], rear at
 * state[0], 310 outputs discarded; each call adds rear into front (mod 2^32) and returns
 * the sum >> 1. */
void lzo_glibc_srand(lzo_glibc_rng *g, uint32_t seed) {
  int32_t word;
  int i;
  if (seed == 0) seed = 1;
  g->ring[0] = seed;
  word = (int32_t)seed;
  for (i = 1; i < 31; ++i) {
    long hi = word / 127773;
    long lo = word % 127773;
    long w = 16807 * lo - 2836 * hi;
    if (w < 0) w += 2147483647;
    word = (int32_t)w;
    g->ring[i] = (uint32_t)word;
  }
  g->f = 3;
  g->r = 0;
  for (i = 0; i < 310; ++i) (void)lzo_glibc_rand(g);
}

int32_t lzo_glibc_rand(lzo_glibc_rng *g) {
  uint32_t v = g->ring[g->f] + g->ring[g->r];
  g->ring[g->f] = v;
  if (++g->f >= 31) {
    g->f = 0;
    ++g->r;
  } else if (++g->r >= 31) {
    g->r = 0;
  }
  return (int32_t)(v >> 1);
}

/* ---------------------------------------------------------------- tree */
typedef struct {
  float maximum, minimum, value_delta_max; /* cminimax.h:17 */
} lzo_minmax;

struct lzo_tree {
  int B, A, cap, ez;
  /* per node [B][cap] */
  int32_t *visit, *to_play, *latent, *batch, *best;
  float *reward, *prior, *value_sum; /* reward == value_prefix for ez */
  int32_t *is_reset;
  /* per root */
  int32_t *legal, *nlegal; /* [B][A], [B] */
  lzo_minmax *mms;
  /* last traverse results */
  int32_t *path;    /* [B][cap] node ids, root first */
  int32_t *pathlen; /* [B] number of nodes on the path */
};

#define NODE(t, i, n) ((size_t)(i) * (size_t)(t)->cap + (size_t)(n))

static void minmax_init(lzo_minmax *m) { /* cminimax.cpp:7-11 */
  m->maximum = LZO_FLOAT_MIN;
  m->minimum = LZO_FLOAT_MAX;
  m->value_delta_max = 0.0f;
}
static void minmax_update(lzo_minmax *m, float v) { /* cminimax.cpp:19-26 */
  if (v > m->maximum) m->maximum = v;
  if (v < m->minimum) m->minimum = v;
}
static float minmax_normalize(const lzo_minmax *m, float v) { /* cminimax.cpp:33-45 */
  float norm = v;
  float delta = m->maximum - m->minimum;
  if (delta > 0) {
    if (delta < m->value_delta_max)
      norm = (norm - m->minimum) / m->value_delta_max;
    else
      norm = (norm - m->minimum) / delta;
  }
  return norm;
}

lzo_tree *lzo_create(int B, int A, int max_sims, int ez) {
  lzo_tree *t = (lzo_tree *)calloc(1, sizeof(lzo_tree));
  size_t n;
  int i;
  t->B = B;
  t->A = A;
  t->cap = 1 + A * (max_sims + 1);
  t->ez = ez;
  n = (size_t)B * t->cap;
  t->visit = calloc(n, 4); t->to_play = calloc(n, 4); t->latent = calloc(n, 4);
  t->batch = calloc(n, 4); t->best = calloc(n, 4); t->reward = calloc(n, 4);
  t->prior = calloc(n, 4); t->value_sum = calloc(n, 4); t->is_reset = calloc(n, 4);
  t->path = calloc(n, 4);
  t->pathlen = calloc(B, 4);
  t->legal = calloc((size_t)B * A, 4);
  t->nlegal = calloc(B, 4);
  t->mms = calloc(B, sizeof(lzo_minmax));
  for (i = 0; i < B; ++i) {
    int a;
    t->nlegal[i] = A;
    for (a = 0; a < A; ++a) t->legal[(size_t)i * A + a] = a;
    minmax_init(&t->mms[i]);
  }
  /* CNode() / CNode(prior, legal): visit 0, value_sum 0, best -1, to_play 0, index -1
   * (ctree_muzero/lib/cnode.cpp:45-79) */
  for (n = 0; n < (size_t)B * t->cap; ++n) {
    t->best[n] = -1;
    t->latent[n] = -1;
    t->batch[n] = -1;
  }
  return t;
}

void lzo_destroy(lzo_tree *t) {
  if (!t) return;
  free(t->visit); free(t->to_play); free(t->latent); free(t->batch); free(t->best);
  free(t->reward); free(t->prior); free(t->value_sum); free(t->is_reset); free(t->path);
  free(t->pathlen); free(t->legal); free(t->nlegal); free(t->mms); free(t);
}

void lzo_set_legal(lzo_tree *t, const int32_t *legal, const int32_t *count) {
  memcpy(t->legal, legal, sizeof(int32_t) * (size_t)t->B * t->A);
  memcpy(t->nlegal, count, sizeof(int32_t) * (size_t)t->B);
}

void lzo_set_delta(lzo_tree *t, float d) { /* CMinMaxStatsList::set_delta, cminimax.cpp:61-65 */
  int i;
  for (i = 0; i < t->B; ++i) t->mms[i].value_delta_max = d;
}

static inline int legal_at(const lzo_tree *t, int i, int node, int j) {
  /* root: the list given to CRoots (cnode.cpp:313-316); other nodes: 0..A-1 (cnode.cpp:101-107) */
  return node == 0 ? t->legal[(size_t)i * t->A + j] : j;
}
static inline int legal_n(const lzo_tree *t, int i, int node) { return node == 0 ? t->nlegal[i] : t->A; }
static inline int child_of(const lzo_tree *t, int i, int node, int a) {
  return 1 + t->A * t->latent[NODE(t, i, node)] + a;
}
static inline float node_value(const lzo_tree *t, size_t k) { /* CNode::value, cnode.cpp:219-235 */
  if (t->visit[k] == 0) return 0.0f;
  return t->value_sum[k] / t->visit[k];
}

/* CNode::expand, ctree_muzero/lib/cnode.cpp:83-147 (ez: value_prefix in place of reward) */
static void expand(lzo_tree *t, int i, int node, int to_play, int latent_index, int batch_index,
                   float reward, const float *logits) {
  size_t k = NODE(t, i, node);
  int n = legal_n(t, i, node), j;
  float policy_max = LZO_FLOAT_MIN, policy_sum = 0.0f;
  float pol[256];
  t->to_play[k] = to_play;
  t->latent[k] = latent_index;
  t->batch[k] = batch_index;
  t->reward[k] = reward;
  for (j = 0; j < n; ++j) {
    int a = legal_at(t, i, node, j);
    if (policy_max < logits[a]) policy_max = logits[a];
  }
  for (j = 0; j < n; ++j) {
    int a = legal_at(t, i, node, j);
    float e = expf(logits[a] - policy_max);
    policy_sum += e;
    pol[a] = e;
  }
  for (j = 0; j < n; ++j) {
    int a = legal_at(t, i, node, j);
    size_t c = NODE(t, i, child_of(t, i, node, a));
    t->prior[c] = pol[a] / policy_sum;
    t->visit[c] = 0; t->value_sum[c] = 0.0f; t->best[c] = -1; t->to_play[c] = 0;
    t->latent[c] = -1; t->batch[c] = -1; t->reward[c] = 0.0f; t->is_reset[c] = 0;
  }
}

/* CRoots::prepare / prepare_no_noise, cnode.cpp:321-358; add_exploration_noise :149-167 */
void lzo_prepare(lzo_tree *t, float f, const float *noises, const float *rewards, const float *logits,
                 const int32_t *to_play) {
  int i, j;
  for (i = 0; i < t->B; ++i) {
    size_t r = NODE(t, i, 0);
    t->visit[r] = 0; t->value_sum[r] = 0.0f; t->best[r] = -1; t->prior[r] = 0.0f; t->is_reset[r] = 0;
    expand(t, i, 0, to_play[i], 0, i, rewards[i], logits + (size_t)i * t->A);
    if (noises) {
      for (j = 0; j < t->nlegal[i]; ++j) {
        size_t c = NODE(t, i, child_of(t, i, 0, t->legal[(size_t)i * t->A + j]));
        float noise = noises[(size_t)i * t->A + j];
        float prior = t->prior[c];
        t->prior[c] = prior * (1 - f) + noise * f;
      }
    }
    t->visit[r] += 1;
    /* a fresh MinMaxStatsList per search (mcts_ctree.py:251-252); value_delta_max kept */
    t->mms[i].maximum = LZO_FLOAT_MIN;
    t->mms[i].minimum = LZO_FLOAT_MAX;
  }
}

/* "true reward" of child c under parent p: mz reward (cnode.cpp:186, :683);
 * ez value_prefix difference with reset (ctree_efficientzero/lib/cnode.cpp:191-195, :786-791) */
static inline float true_reward(const lzo_tree *t, size_t p, size_t c) {
  if (!t->ez) return t->reward[c];
  if (t->is_reset[p] == 1) return t->reward[c];
  return t->reward[c] - t->reward[p];
}

/* CNode::compute_mean_q, cnode.cpp:169-203 */
static float compute_mean_q(const lzo_tree *t, int i, int node, int is_root, float parent_q, float disc) {
  size_t p = NODE(t, i, node);
  float total_unsigned_q = 0.0f;
  int total_visits = 0, j, n = legal_n(t, i, node);
  float mean_q;
  for (j = 0; j < n; ++j) {
    size_t c = NODE(t, i, child_of(t, i, node, legal_at(t, i, node, j)));
    if (t->visit[c] > 0) {
      float qsa = true_reward(t, p, c) + disc * node_value(t, c);
      total_unsigned_q += qsa;
      total_visits += 1;
    }
  }
  if (is_root && total_visits > 0)
    mean_q = total_unsigned_q / total_visits;
  else
    mean_q = (parent_q + total_unsigned_q) / (total_visits + 1);
  return mean_q;
}

/* cucb_score, cnode.cpp:655-699 (ez: :756-814) */
static float ucb_score(const lzo_tree *t, int i, size_t p, size_t c, float parent_mean_q, float total_children_visit_counts,
                       float pb_c_base, float pb_c_init, float disc, int players) {
  float pb_c, prior_score, value_score;
  pb_c = logf((total_children_visit_counts + pb_c_base + 1) / pb_c_base) + pb_c_init;
  pb_c *= (sqrtf(total_children_visit_counts) / (t->visit[c] + 1));
  prior_score = pb_c * t->prior[c];
  if (t->visit[c] == 0) {
    value_score = parent_mean_q;
  } else {
    float tr = true_reward(t, p, c);
    if (players == 1)
      value_score = tr + disc * node_value(t, c);
    else
      value_score = tr + disc * (-node_value(t, c));
  }
  value_score = minmax_normalize(&t->mms[i], value_score);
  if (value_score < 0) value_score = 0;
  if (value_score > 1) value_score = 1;
  return prior_score + value_score;
}

/* cselect_child, cnode.cpp:551-596: order-dependent 1e-6 tie list, exactly one rand() */
static int32_t draw_next_fwd(void *d, int root, int level);
static int select_child(const lzo_tree *t, int i, int node, int pb_c_base, float pb_c_init, float disc,
                        float mean_q, int players, void *dr, int level) {
  size_t p = NODE(t, i, node);
  float max_score = LZO_FLOAT_MIN;
  const float epsilon = 0.000001f;
  int lst[256], nl = 0, j, n = legal_n(t, i, node), action = 0;
  for (j = 0; j < n; ++j) {
    int a = legal_at(t, i, node, j);
    size_t c = NODE(t, i, child_of(t, i, node, a));
    float s = ucb_score(t, i, p, c, mean_q, (float)(t->visit[p] - 1), (float)pb_c_base, pb_c_init, disc, players);
    if (max_score < s) {
      max_score = s;
      nl = 0;
      lst[nl++] = a;
    } else if (s >= max_score - epsilon) {
      lst[nl++] = a;
    }
  }
  if (nl > 0) action = lst[draw_next_fwd(dr, i, level) % nl];
  return action;
}

/* Philox4x32-10 (Salmon et al., SC'11), for the LZM_RNG_FAST tie-break stream:
 * draw(root i, level l) = philox(ctr = {l, i, 0, 0}, key = {seed, 0x4c5a4d43}).x >> 1 */
void lzo_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
  uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3], k0 = key_in[0], k1 = key_in[1];
  int r;
  for (r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0, hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* draw source: glibc stream (serial over roots) or philox per (root, level) */
typedef struct {
  int fast;
  uint32_t seed;
  lzo_glibc_rng g;
} lzo_draws;

static int32_t draw_next(lzo_draws *d, int root, int level) {
  if (!d->fast) return lzo_glibc_rand(&d->g);
  {
    uint32_t ctr[4] = {(uint32_t)level, (uint32_t)root, 0u, 0u}, key[2] = {d->seed, 0x4c5a4d43u}, o[4];
    lzo_philox4x32_10(ctr, key, o);
    return (int32_t)(o[0] >> 1);
  }
}

/* cbatch_traverse, cnode.cpp:755-824 */
static void traverse_impl(lzo_tree *t, int pb_c_base, float pb_c_init, float disc, lzo_draws *dr, const int32_t *vtp_in,
                          int32_t *out_x, int32_t *out_y, int32_t *out_a, int32_t *out_vtp, int32_t *out_len) {
  int i, players, largest = vtp_in[0], last_action = -1;
  float parent_q = 0.0f; /* declared once per call and carried across roots, cnode.cpp:773 */
  for (i = 1; i < t->B; ++i)
    if (vtp_in[i] > largest) largest = vtp_in[i];
  players = (largest == -1) ? 1 : 2;
  for (i = 0; i < t->B; ++i) {
    int node = 0, is_root = 1, search_len = 0, vtp = vtp_in[i];
    int32_t *path = t->path + (size_t)i * t->cap;
    int np = 0;
    path[np++] = 0;
    while (t->latent[NODE(t, i, node)] >= 0) { /* expanded(): children exist */
      float mean_q = compute_mean_q(t, i, node, is_root, parent_q, disc);
      int action;
      is_root = 0;
      parent_q = mean_q;
      action = select_child(t, i, node, pb_c_base, pb_c_init, disc, mean_q, players, dr, search_len);
      if (players > 1) vtp = (vtp == 1) ? 2 : 1;
      t->best[NODE(t, i, node)] = action;
      node = child_of(t, i, node, action);
      last_action = action;
      path[np++] = node;
      search_len += 1;
    }
    t->pathlen[i] = np;
    {
      size_t par = NODE(t, i, path[np - 2]);
      out_x[i] = t->latent[par];
      out_y[i] = t->batch[par];
    }
    out_a[i] = last_action;
    out_len[i] = search_len;
    out_vtp[i] = vtp;
  }
}

static int32_t draw_next_fwd(void *d, int root, int level) { return draw_next((lzo_draws *)d, root, level); }

void lzo_traverse(lzo_tree *t, int pb_c_base, float pb_c_init, float disc, uint32_t seed, const int32_t *vtp_in,
                  int32_t *out_x, int32_t *out_y, int32_t *out_a, int32_t *out_vtp, int32_t *out_len) {
  lzo_draws d;
  d.fast = 0;
  d.seed = seed;
  lzo_glibc_srand(&d.g, seed); /* srand(tv_usec), common_lib/utils.cpp:25 */
  traverse_impl(t, pb_c_base, pb_c_init, disc, &d, vtp_in, out_x, out_y, out_a, out_vtp, out_len);
}

void lzo_traverse_fast(lzo_tree *t, int pb_c_base, float pb_c_init, float disc, uint32_t seed, const int32_t *vtp_in,
                       int32_t *out_x, int32_t *out_y, int32_t *out_a, int32_t *out_vtp, int32_t *out_len) {
  lzo_draws d;
  d.fast = 1;
  d.seed = seed;
  traverse_impl(t, pb_c_base, pb_c_init, disc, &d, vtp_in, out_x, out_y, out_a, out_vtp, out_len);
}

/* cbackpropagate, mz: cnode.cpp:419-478; ez: ctree_efficientzero/lib/cnode.cpp:482-575 */
static void backpropagate(lzo_tree *t, int i, int to_play, float value, float disc) {
  const int32_t *path = t->path + (size_t)i * t->cap;
  int np = t->pathlen[i], j;
  lzo_minmax *m = &t->mms[i];
  float b = value;
  for (j = np - 1; j >= 0; --j) {
    size_t k = NODE(t, i, path[j]);
    float tr;
    int reset = 0;
    if (to_play == -1 || t->to_play[k] == to_play)
      t->value_sum[k] += b;
    else
      t->value_sum[k] += -b;
    t->visit[k] += 1;
    if (!t->ez) {
      tr = t->reward[k];
      if (to_play == -1) {
        minmax_update(m, tr + disc * node_value(t, k));
        b = tr + disc * b;
      } else {
        minmax_update(m, tr + disc * -node_value(t, k));
        if (t->to_play[k] == to_play)
          b = -tr + disc * b;
        else
          b = tr + disc * b;
      }
    } else {
      float pvp = 0.0f;
      if (j >= 1) {
        size_t pk = NODE(t, i, path[j - 1]);
        pvp = t->reward[pk];
        reset = t->is_reset[pk];
      }
      tr = t->reward[k] - pvp;
      minmax_update(m, tr + disc * node_value(t, k));
      if (reset == 1) tr = t->reward[k];
      if (to_play == -1 || t->to_play[k] != to_play)
        b = tr + disc * b;
      else
        b = -tr + disc * b;
    }
  }
}

/* cbatch_backpropagate, cnode.cpp:480-500 (ez :577-601 adds is_reset) */
void lzo_backprop(lzo_tree *t, int cur, float disc, const float *rewards, const float *values, const float *logits,
                  const int32_t *is_reset, const int32_t *to_play) {
  int i;
  if (1 + t->A * (cur + 1) > t->cap) {
    fprintf(stderr, "lzo_backprop: latent index %d exceeds capacity\n", cur);
    abort();
  }
  for (i = 0; i < t->B; ++i) {
    const int32_t *path = t->path + (size_t)i * t->cap;
    int leaf = path[t->pathlen[i] - 1];
    expand(t, i, leaf, to_play[i], cur, i, rewards[i], logits + (size_t)i * t->A);
    if (t->ez && is_reset) t->is_reset[NODE(t, i, leaf)] = is_reset[i];
    backpropagate(t, i, to_play[i], values[i], disc);
  }
}

/* CRoots::get_distributions, cnode.cpp:387-403 / get_children_distribution :259-277 */
void lzo_get_distributions(const lzo_tree *t, int32_t *out) {
  int i, j;
  for (i = 0; i < t->B; ++i) {
    for (j = 0; j < t->A; ++j) out[(size_t)i * t->A + j] = -1;
    if (t->latent[NODE(t, i, 0)] < 0) continue;
    for (j = 0; j < t->nlegal[i]; ++j)
      out[(size_t)i * t->A + j] = t->visit[NODE(t, i, child_of(t, i, 0, t->legal[(size_t)i * t->A + j]))];
  }
}

void lzo_get_values(const lzo_tree *t, float *out) { /* CRoots::get_values, cnode.cpp:405-417 */
  int i;
  for (i = 0; i < t->B; ++i) out[i] = node_value(t, NODE(t, i, 0));
}

/* CRoots::get_trajectories / CNode::get_trajectory, cnode.cpp:237-257, :369-385 */
int lzo_get_trajectories(const lzo_tree *t, int32_t *out, int tmax) {
  int i, longest = 0;
  for (i = 0; i < t->B; ++i) {
    int node = 0, n = 0, ba = t->best[NODE(t, i, 0)];
    while (ba >= 0) {
      if (n < tmax) out[(size_t)i * tmax + n] = ba;
      n++;
      node = child_of(t, i, node, ba);
      ba = t->best[NODE(t, i, node)];
    }
    if (n > longest) longest = n;
    for (; n < tmax; ++n) out[(size_t)i * tmax + n] = -1;
  }
  return longest;
}

/* ---------------------------------------------------------------- CPU baseline driver */
typedef struct {
  int B, A, S, searches;
  uint32_t seed;
  double secs;
} bench_arg;

static uint32_t xs32(uint32_t *s) {
  uint32_t x = *s;
  x ^= x << 13; x ^= x >> 17; x ^= x << 5;
  return *s = x;
}
static float unitf(uint32_t *s) { return (float)((xs32(s) >> 8) * (1.0 / 16777216.0)) * 2.0f - 1.0f; }

static void *bench_worker(void *p) {
  bench_arg *a = (bench_arg *)p;
  int B = a->B, A = a->A, S = a->S, it, k, i;
  lzo_tree *t = lzo_create(B, A, S, 0);
  float *noises = malloc(sizeof(float) * B * A), *logits = malloc(sizeof(float) * B * A);
  float *rw = malloc(sizeof(float) * B), *val = malloc(sizeof(float) * B), *r0 = calloc(B, sizeof(float));
  int32_t *tp = malloc(4 * B), *x = malloc(4 * B), *y = malloc(4 * B), *ac = malloc(4 * B), *vtp = malloc(4 * B),
          *len = malloc(4 * B);
  uint32_t s = a->seed * 2654435761u + 1u;
  struct timespec t0, t1;
  for (i = 0; i < B; ++i) tp[i] = -1;
  for (i = 0; i < B * A; ++i) { noises[i] = 1.0f / A; logits[i] = unitf(&s); }
  lzo_set_delta(t, 0.01f);
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (it = 0; it < a->searches; ++it) {
    lzo_prepare(t, 0.25f, noises, r0, logits, tp);
    for (k = 0; k < S; ++k) {
      lzo_traverse(t, 19652, 1.25f, 0.997f, (a->seed + k) % 1000000u, tp, x, y, ac, vtp, len);
      for (i = 0; i < B; ++i) { rw[i] = unitf(&s) * 0.5f; val[i] = unitf(&s); }
      for (i = 0; i < B * A; ++i) logits[i] = unitf(&s);
      lzo_backprop(t, k + 1, 0.997f, rw, val, logits, NULL, vtp);
    }
  }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  a->secs = (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
  lzo_destroy(t);
  free(noises); free(logits); free(rw); free(val); free(r0); free(tp); free(x); free(y); free(ac); free(vtp); free(len);
  return NULL;
}

/* ---------------------------------------------------------------- diagnostics (tests only) */
int lzo_get_path_actions(const lzo_tree *t, int i, int32_t *out, int cap) {
  const int32_t *path = t->path + (size_t)i * t->cap;
  int np = t->pathlen[i], l, n = 0;
  for (l = 0; l + 1 < np && n < cap; ++l) {
    int parent_latent = t->latent[NODE(t, i, path[l])];
    out[n++] = path[l + 1] - 1 - t->A * parent_latent; /* child_of inverted */
  }
  return n;
}

int lzo_path_scores(const lzo_tree *t, int i, int pb_c_base, float pb_c_init, float disc, int players,
                    const int32_t *actions, int n, float *out) {
  int node = 0, is_root = 1, lvl = 0, a, j;
  float parent_q = 0.0f;
  while (lvl <= n && t->latent[NODE(t, i, node)] >= 0) {
    size_t p = NODE(t, i, node);
    float mean_q = compute_mean_q(t, i, node, is_root, parent_q, disc);
    is_root = 0;
    parent_q = mean_q;
    for (a = 0; a < t->A; ++a) out[(size_t)lvl * t->A + a] = -INFINITY;
    for (j = 0; j < legal_n(t, i, node); ++j) {
      a = legal_at(t, i, node, j);
      out[(size_t)lvl * t->A + a] = ucb_score(t, i, p, NODE(t, i, child_of(t, i, node, a)), mean_q,
                                              (float)(t->visit[p] - 1), (float)pb_c_base, pb_c_init, disc, players);
    }
    if (lvl == n) return lvl + 1;
    node = child_of(t, i, node, actions[lvl]);
    lvl += 1;
  }
  return lvl;
}

double lzo_bench_tree_only(int B, int A, int S, int threads, int searches, uint32_t seed) {
  pthread_t th[256];
  bench_arg args[256];
  int w, base = 0;
  struct timespec t0, t1;
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  if (threads > B) threads = B;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (w = 0; w < threads; ++w) {
    int nb = B / threads + (w < B % threads ? 1 : 0);
    args[w].B = nb; args[w].A = A; args[w].S = S; args[w].searches = searches; args[w].seed = seed + 7919u * w;
    base += nb;
    pthread_create(&th[w], NULL, bench_worker, &args[w]);
  }
  for (w = 0; w < threads; ++w) pthread_join(th[w], NULL);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  (void)base;
  return (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
}

/* ---------------------------------------------------------------- expf exhaustive checker */
typedef struct {
  uint32_t first;
  int64_t lo, hi;
  const float *got;
  long bad;
} expf_arg;

static void *expf_worker(void *p) {
  expf_arg *a = (expf_arg *)p;
  int64_t k;
  for (k = a->lo; k < a->hi; ++k) {
    uint32_t u = a->first + (uint32_t)k;
    float x, e;
    memcpy(&x, &u, 4);
    e = expf(x);
    if (memcmp(&e, &a->got[k], 4) != 0) a->bad++;
  }
  return NULL;
}

/* Counts k in [0,n) where host libm expf(bits(first+k)) differs bitwise from got[k]. */
long lzo_expf_mismatches(uint32_t first, int64_t n, const float *got, int threads) {
  pthread_t th[64];
  expf_arg args[64];
  int w;
  long bad = 0;
  if (threads < 1) threads = 1;
  if (threads > 64) threads = 64;
  for (w = 0; w < threads; ++w) {
    args[w].first = first;
    args[w].lo = n * w / threads;
    args[w].hi = n * (w + 1) / threads;
    args[w].got = got;
    args[w].bad = 0;
    pthread_create(&th[w], NULL, expf_worker, &args[w]);
  }
  for (w = 0; w < threads; ++w) {
    pthread_join(th[w], NULL);
    bad += args[w].bad;
  }
  return bad;
}
