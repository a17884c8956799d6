"""Reference-vs-restatement CPU calibration (BASELINE.md CPU-baseline plan step 2).

Runs in the BUILD CONTAINER only, where the reference's own ctree can be compiled from
/root/reference (oracle/build_ref.sh -> oracle/_ref, git-ignored and gpurun-ignored: the reference
never travels to the GPU box). On the GPU box bench.py times the oracle's bit-exact restatement
("port"); this script measures, on the same host, how the two compare, so the box's port numbers
can be read as reference numbers:

  tree_only : the reference search loop's tree calls only (mcts_ctree.py:255-321 with the network
              replaced by precomputed response lists): Roots.prepare + S x (batch_traverse,
              batch_backpropagate) through the reference's Cython module on Python lists, against
              the same loop over the oracle (ctypes, numpy arrays). 1 core, as the reference ctree.
  ref_arch  : the whole reference search architecture on the CPU (bench.py cpu_reference_search:
              host tree + MuZeroModelMLP on torch-CPU + InverseScalarTransform + list glue) with the
              reference's ctree and with the oracle, same threads.

  az        : config 4, the per-board AlphaZero search with per-leaf network calls over the reference's
              mcts_alphazero and over the port (oracle/az_oracle.py), 1 thread (--az: this entry only).

Writes profiles/cpu_calibration.json with time ratios reference / port (> 1: the port is faster).

    bash oracle/build_ref.sh && python tools/cpu_calibration.py [--az]
"""
import glob
import importlib.util
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402
from oracle.oracle import OracleTree  # noqa: E402


def load_ref():
    paths = sorted(glob.glob(os.path.join(REPO, "oracle", "_ref", "mz_tree*.so")))
    if not paths:
        sys.exit("oracle/_ref missing: run oracle/build_ref.sh first (build container only)")
    spec = importlib.util.spec_from_file_location("mz_tree", paths[0])
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def scripted(B, S, A, seed=0):
    rng = np.random.default_rng(seed)
    return dict(noises=rng.dirichlet([0.3] * A, size=B).astype(np.float32),
                logits0=rng.normal(size=(B, A)).astype(np.float32),
                r=(rng.normal(size=(S, B)) * 0.5).astype(np.float32), v=rng.normal(size=(S, B)).astype(np.float32),
                p=rng.normal(size=(S, B, A)).astype(np.float32))


def tree_only_ref(mod, tab, B, S, A, reps):
    legal = [list(range(A)) for _ in range(B)]
    tp = [-1] * B
    lists = dict(noises=tab["noises"].tolist(), logits0=tab["logits0"].tolist(), r=[x.tolist() for x in tab["r"]],
                 v=[x.tolist() for x in tab["v"]], p=[x.tolist() for x in tab["p"]])
    t0 = time.perf_counter()
    for it in range(reps):
        roots = mod.Roots(B, legal)
        roots.prepare(0.25, lists["noises"], [0.0] * B, lists["logits0"], tp)
        mms = mod.MinMaxStatsList(B)
        mms.set_delta(0.01)
        for k in range(S):
            results = mod.ResultsWrapper(num=B)
            x, y, a, vtp = mod.batch_traverse(roots, 19652, 1.25, 0.997, mms, results, tp)
            mod.batch_backpropagate(k + 1, 0.997, lists["r"][k], lists["v"][k], lists["p"][k], mms, results, vtp)
        roots.get_distributions()
    return time.perf_counter() - t0


def tree_only_port(tab, B, S, A, reps):
    tp = np.full(B, -1, np.int32)
    t0 = time.perf_counter()
    for it in range(reps):
        t = OracleTree(B, A, S)
        t.set_delta(np.float32(0.01))
        t.prepare(np.float32(0.25), tab["noises"], np.zeros(B, np.float32), tab["logits0"], tp)
        for k in range(S):
            x, y, a, vtp, _ = t.traverse(19652, np.float32(1.25), np.float32(0.997), k, tp)
            t.backprop(k + 1, np.float32(0.997), tab["r"][k], tab["v"][k], tab["p"][k], vtp)
        t.distributions()
    return time.perf_counter() - t0


def ref_arch_ref(mod, B, S, model_cpu, secs, threads):
    """bench.cpu_reference_search with the reference's compiled ctree in place of the oracle"""
    torch.set_num_threads(threads)
    rng = np.random.default_rng(0)
    obs = torch.from_numpy(rng.normal(size=(B, 4)).astype(np.float32))
    support = torch.arange(-300, 301, dtype=torch.float64).unsqueeze(0)

    def inv(logits):
        p = torch.softmax(logits, dim=1)
        v = p.mul_(support).sum(1, keepdim=True)
        tmp = (torch.sqrt(1 + 4 * 0.001 * (torch.abs(v) + 1 + 0.001)) - 1) / (2 * 0.001)
        return (torch.sign(v) * (tmp * tmp - 1)).float()

    legal = [[0, 1] for _ in range(B)]
    to_play = [-1] * B
    n, t0 = 0, time.perf_counter()
    with torch.no_grad():
        while True:
            out = model_cpu.initial_inference(obs)
            roots = mod.Roots(B, legal)
            noises = rng.dirichlet([0.3, 0.3], size=B).astype(np.float32).tolist()
            roots.prepare(0.25, noises, [0.0] * B, out.policy_logits.numpy().tolist(), to_play)
            pool = [out.latent_state.numpy()]
            mms = mod.MinMaxStatsList(B)
            mms.set_delta(0.01)
            for k in range(S):
                results = mod.ResultsWrapper(num=B)
                x, y, a, vtp = mod.batch_traverse(roots, 19652, 1.25, 0.997, mms, results, to_play)
                lat = torch.from_numpy(np.asarray([pool[ix][iy] for ix, iy in zip(x, y)]))
                o = model_cpu.recurrent_inference(lat, torch.from_numpy(np.asarray(a)).long())
                pool.append(o.latent_state.numpy())
                mod.batch_backpropagate(k + 1, 0.997, inv(o.reward).numpy().reshape(-1).tolist(),
                                        inv(o.value).numpy().reshape(-1).tolist(), o.policy_logits.numpy().tolist(),
                                        mms, results, vtp)
            n += 1
            el = time.perf_counter() - t0
            if el >= secs:
                return n * B * S / el, n, el


def az_calibration(secs=6.0):
    """config 4: the reference's compiled mcts_alphazero (oracle/_ref) vs the port (oracle/az_oracle.py), each
    driving the same AlphaZeroModel on torch-CPU per leaf (bench.cpu_baseline_az's loop), 1 thread, the same
    boards; returns the "az" entry (time ratio reference / port)"""
    paths = sorted(glob.glob(os.path.join(REPO, "oracle", "_ref", "mcts_alphazero*.so")))
    if not paths:
        sys.exit("oracle/_ref missing: run oracle/build_ref.sh first (build container only)")
    spec = importlib.util.spec_from_file_location("mcts_alphazero", paths[0])
    az = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(az)
    from lightzero_amd.model_az import tictactoe_alphazero_model
    from oracle.tictactoe import SimTicTacToe
    torch.set_num_threads(1)
    torch.manual_seed(0)
    net = tictactoe_alphazero_model().eval()
    boards, starts = bench.az_boards(64, 0)
    S = 100

    def pv(e):
        legal = e.legal_actions
        _, scaled = e.current_state()
        with torch.no_grad():
            probs, value = net.compute_policy_value(torch.from_numpy(scaled).float().unsqueeze(0))
        return dict(zip(legal, probs.squeeze(0)[legal].numpy())), value.item()

    def ref_rate():
        mcts = az.MCTS(9, S, 19652, 1.25, 0.3, 0.25, SimTicTacToe(scale=True))
        n, t0 = 0, time.perf_counter()
        while True:
            b, st = boards[n % len(boards)], starts[n % len(boards)]
            mcts.get_next_action(dict(start_player_index=int(st), init_state=b.reshape(3, 3).astype(np.int32),
                                      katago_policy_init=False, katago_game_state=None), pv, 1.0, True)
            n += 1
            el = time.perf_counter() - t0
            if el >= secs:
                return n * S / el

    vr, vp = [], []
    for _ in range(2):
        vr.append(ref_rate())
        vp.append(bench.cpu_baseline_az(net, boards, starts, S, secs)["value"])
    return {"ref_sims_per_s": round(max(vr), 1), "port_sims_per_s": round(max(vp), 1), "threads": 1,
            "loop": "per-board search, AlphaZeroModel on torch-CPU called per leaf (policy/alphazero.py:371-380)",
            "ref_over_port_time": round(max(vp) / max(vr), 3)}


def main():
    if "--az" in sys.argv:  # refresh the config-4 entry only
        out = os.path.join(REPO, "profiles", "cpu_calibration.json")
        with open(out) as f:
            res = json.load(f)
        res["az"] = az_calibration()
        with open(out, "w") as f:
            json.dump(res, f, indent=1)
        print(json.dumps(res["az"], indent=1))
        return
    mod = load_ref()
    B, S, A = 256, 50, 2
    tab = scripted(B, S, A)
    res = {"host": bench.host_cpu_info(), "shape": {"B": B, "S": S, "A": A}}
    # tree only, 1 core: alternate the two, best of 3 rounds
    tr, tp = [], []
    for _ in range(3):
        tr.append(tree_only_ref(mod, tab, B, S, A, 4))
        tp.append(tree_only_port(tab, B, S, A, 4))
    res["tree_only"] = {"ref_sims_per_s": round(4 * B * S / min(tr), 1), "port_sims_per_s": round(4 * B * S / min(tp), 1),
                        "port_c_driver_sims_per_s": round(bench.cpu_tree_only(B, A, S, 1, 3.0)[0], 1),
                        "loop": "Roots.prepare + S x (batch_traverse, batch_backpropagate), precomputed responses"}
    res["ref_over_port_time_tree_only"] = round(min(tr) / min(tp), 3)
    # whole reference architecture on the CPU
    threads = min(8, os.cpu_count() or 1)
    model_cpu = bench.build_model(torch.device("cpu"), False, seed=0)
    vr, vp = [], []
    for _ in range(2):
        vr.append(ref_arch_ref(mod, B, S, model_cpu, 6.0, threads)[0])
        vp.append(bench.cpu_reference_search(B, S, model_cpu, 6.0, threads)[0])
    res["ref_arch"] = {"ref_sims_per_s": round(max(vr), 1), "port_sims_per_s": round(max(vp), 1),
                       "threads": threads, "network": "MuZeroModelMLP on torch-CPU"}
    res["ref_over_port_time_ref_arch"] = round(max(vp) / max(vr), 3)
    res["az"] = az_calibration()
    out = os.path.join(REPO, "profiles", "cpu_calibration.json")
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
