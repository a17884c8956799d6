"""ctypes wrapper around oracle/liblzoracle.so — the CPU restatement of LightZero's ctree.

TEST INFRASTRUCTURE ONLY: imported by tests/, ``__graft_entry__.smoke()`` and bench.py's
``cpu_baseline`` leg, as the checker / CPU baseline. The product package ``lightzero_amd``
never imports this module.

``replay_transcript`` restates the driving loop of ``MuZeroMCTSCtree.search``
(/root/reference/lzero/mcts/tree_search/mcts_ctree.py:255-321) over a golden transcript:
the network is replaced by the recorded responses, and every request the tree issues is
compared with the recorded one.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liblzoracle.so")

_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
_u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")
_lib = None


def build():
    import subprocess
    subprocess.check_call(["make", "-s", "-C", HERE, "liblzoracle.so"])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.lzo_create.restype = ctypes.c_void_p
        L.lzo_create.argtypes = [ctypes.c_int] * 4
        L.lzo_destroy.argtypes = [ctypes.c_void_p]
        L.lzo_set_legal.argtypes = [ctypes.c_void_p, _i32p, _i32p]
        L.lzo_set_delta.argtypes = [ctypes.c_void_p, ctypes.c_float]
        L.lzo_prepare.argtypes = [ctypes.c_void_p, ctypes.c_float, ctypes.c_void_p, _f32p, _f32p, _i32p]
        L.lzo_traverse.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_float, ctypes.c_uint32,
                                   _i32p, _i32p, _i32p, _i32p, _i32p, _i32p]
        L.lzo_traverse_fast.argtypes = L.lzo_traverse.argtypes
        L.lzo_philox4x32_10.argtypes = [_u32p, _u32p, _u32p]
        L.lzo_backprop.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_float, _f32p, _f32p, _f32p,
                                   ctypes.c_void_p, _i32p]
        L.lzo_get_distributions.argtypes = [ctypes.c_void_p, _i32p]
        L.lzo_get_values.argtypes = [ctypes.c_void_p, _f32p]
        L.lzo_get_trajectories.restype = ctypes.c_int
        L.lzo_get_trajectories.argtypes = [ctypes.c_void_p, _i32p, ctypes.c_int]
        L.lzo_glibc_srand.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        L.lzo_glibc_rand.restype = ctypes.c_int32
        L.lzo_glibc_rand.argtypes = [ctypes.c_void_p]
        L.lzo_expf_mismatches.restype = ctypes.c_long
        L.lzo_expf_mismatches.argtypes = [ctypes.c_uint32, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int]
        L.lzo_get_path_actions.restype = ctypes.c_int
        L.lzo_get_path_actions.argtypes = [ctypes.c_void_p, ctypes.c_int, _i32p, ctypes.c_int]
        L.lzo_path_scores.restype = ctypes.c_int
        L.lzo_path_scores.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_float,
                                      ctypes.c_int, _i32p, ctypes.c_int, _f32p]
        L.lzo_bench_tree_only.restype = ctypes.c_double
        L.lzo_bench_tree_only.argtypes = [ctypes.c_int] * 5 + [ctypes.c_uint32]
        _lib = L
    return _lib


def philox4x32_10(ctr, key):
    out = np.zeros(4, np.uint32)
    lib().lzo_philox4x32_10(np.ascontiguousarray(ctr, np.uint32), np.ascontiguousarray(key, np.uint32), out)
    return out


def glibc_rand_stream(seed, n):
    L = lib()
    state = ctypes.create_string_buffer(31 * 4 + 8)
    L.lzo_glibc_srand(state, seed)
    return np.array([L.lzo_glibc_rand(state) for _ in range(n)], np.int64)


class OracleTree:
    """One batch of roots (CRoots + CMinMaxStatsList + CSearchResults of the reference)."""

    def __init__(self, num_roots, action_space, max_sims, ez=False, fast_rng=False):
        self.B, self.A = num_roots, action_space
        self.fast_rng = fast_rng
        self._h = lib().lzo_create(num_roots, action_space, max_sims, int(ez))

    def __del__(self):
        if getattr(self, "_h", None):
            lib().lzo_destroy(self._h)
            self._h = None

    def set_legal(self, legal_actions, legal_count):
        lib().lzo_set_legal(self._h, np.ascontiguousarray(legal_actions, np.int32),
                            np.ascontiguousarray(legal_count, np.int32))

    def set_delta(self, d):
        lib().lzo_set_delta(self._h, d)

    def prepare(self, noise_weight, noises, rewards, logits, to_play):
        nz = None if noises is None else np.ascontiguousarray(noises, np.float32)
        lib().lzo_prepare(self._h, noise_weight, None if nz is None else nz.ctypes.data,
                          np.ascontiguousarray(rewards, np.float32), np.ascontiguousarray(logits, np.float32),
                          np.ascontiguousarray(to_play, np.int32))
        self._keep = nz

    def traverse(self, pb_c_base, pb_c_init, discount, seed, virtual_to_play):
        B = self.B
        outs = [np.zeros(B, np.int32) for _ in range(5)]
        fn = lib().lzo_traverse_fast if self.fast_rng else lib().lzo_traverse
        fn(self._h, int(pb_c_base), pb_c_init, discount, int(seed),
                           np.ascontiguousarray(virtual_to_play, np.int32), *outs)
        return tuple(outs)  # x, y, action, vtp, search_len

    def backprop(self, cur, discount, rewards, values, logits, to_play, is_reset=None):
        rs = None if is_reset is None else np.ascontiguousarray(is_reset, np.int32)
        lib().lzo_backprop(self._h, cur, discount, np.ascontiguousarray(rewards, np.float32),
                           np.ascontiguousarray(values, np.float32), np.ascontiguousarray(logits, np.float32),
                           None if rs is None else rs.ctypes.data, np.ascontiguousarray(to_play, np.int32))

    def distributions(self):
        out = np.zeros((self.B, self.A), np.int32)
        lib().lzo_get_distributions(self._h, out)
        return out

    def values(self):
        out = np.zeros(self.B, np.float32)
        lib().lzo_get_values(self._h, out)
        return out

    def path_actions(self, i):
        """root i's last traverse path as actions (diagnostics)"""
        out = np.zeros(self.B * 4 + 64, np.int32)
        n = lib().lzo_get_path_actions(self._h, int(i), out, out.shape[0])
        return out[:n].copy()

    def path_scores(self, i, actions, pb_c_base=19652, pb_c_init=1.25, discount=0.997, players=1):
        """the pUCT scores [levels, A] cselect_child computes along root i's walk down `actions`
        (diagnostics; -inf where an action is not legal)"""
        acts = np.ascontiguousarray(actions, np.int32)
        out = np.zeros((len(acts) + 1, self.A), np.float32)
        n = lib().lzo_path_scores(self._h, int(i), int(pb_c_base), np.float32(pb_c_init), np.float32(discount),
                                  int(players), acts, len(acts), out)
        return out[:n]

    def trajectories(self, tmax=64):
        out = np.zeros((self.B, tmax), np.int32)
        lib().lzo_get_trajectories(self._h, out, tmax)
        return out


def legal_from_mask(mask):
    B, A = mask.shape
    legal = np.full((B, A), -1, np.int32)
    cnt = np.zeros(B, np.int32)
    for i in range(B):
        idx = np.nonzero(mask[i])[0]
        legal[i, :len(idx)] = idx
        cnt[i] = len(idx)
    return legal, cnt


def load_transcript(path):
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def replay_transcript(tr, tree_factory=None, check=True):
    """Replay a golden transcript through a tree object with the OracleTree interface.

    Returns a dict of mismatches (empty when everything is bit-exact)."""
    B, S, A, players, noise, ez, horizon = [int(v) for v in tr["meta"]]
    pb_c_base, pb_c_init, disc, vdm, nw = [float(v) for v in tr["consts"]]
    t = (tree_factory or OracleTree)(B, A, S, ez=bool(ez))
    legal, cnt = legal_from_mask(tr["legal_mask"])
    t.set_legal(legal, cnt)
    t.set_delta(np.float32(vdm))
    t.prepare(np.float32(nw), tr["noises"] if noise else None, tr["root_reward"], tr["root_logits"], tr["to_play"])
    bad = {}
    for k in range(S):
        x, y, a, vtp, slen = t.traverse(pb_c_base, np.float32(pb_c_init), np.float32(disc), int(tr["seeds"][k]),
                                        tr["to_play"])
        for name, got in (("x", x), ("y", y), ("a", a), ("vtp", vtp), ("len", slen)):
            exp = tr["req_" + name][k]
            if not np.array_equal(got, exp):
                bad.setdefault("req_" + name, []).append(k)
        t.backprop(k + 1, np.float32(disc), tr["resp_reward"][k], tr["resp_value"][k], tr["resp_logits"][k],
                   vtp, tr["resp_is_reset"][k] if ez else None)
    dist = t.distributions()
    if not np.array_equal(dist, tr["out_dist"]):
        bad["dist"] = int((dist != tr["out_dist"]).sum())
    vals = t.values()
    if not np.array_equal(vals, tr["out_values"]):
        bad["values_maxdiff"] = float(np.abs(vals - tr["out_values"]).max())
    traj = t.trajectories(max(64, tr["out_traj"].shape[1]))
    T = tr["out_traj"].shape[1]
    if not (np.array_equal(traj[:, :T], tr["out_traj"]) and (traj[:, T:] == -1).all()):
        bad["traj"] = True
    return bad
