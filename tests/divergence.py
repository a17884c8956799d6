"""Test helper: where two searches of the same roots part ways (network-in-the-loop divergence).

Two GPU searches over the same roots, seeds and weights that differ only in how the network rounds
(the fused kernel vs the PyTorch module, or split-bf16 vs exact-f32 trunks) make identical tree
requests until some simulation k at which one root's walk picks a different child. Each search is
replayed through the oracle (oracle/lz_oracle.c, pinned to the reference ctree) with the network
outputs that search recorded — reproducing each GPU tree exactly — and at every root's first divergent
simulation the two oracle trees are asked for the pUCT scores cselect_child saw along each walk
(OracleTree.path_scores). The first level where the walks differ is classified:

  near_tie     the two actions' scores differ by at most `tau` in both trees — float rounding of the
               network outputs moved a near-tie across (cnode.cpp:551-596's 1e-6 epsilon included);
  draw_shift   both actions are in the epsilon tie list in both trees and the choice differs: the
               tie was broken by rand() at a different position of the batch-serial glibc stream,
               because an earlier root of the same simulation (or an earlier simulation) already
               diverged in depth (cbatch_traverse draws one rand() per level over all roots in order,
               cnode.cpp:755-824);
  unexplained  anything else (a bug: must be zero).
Also reported: the typical gap between the chosen child and the runner-up over every level of every
walk, for scale.
"""
import json
import os

import numpy as np

from oracle.oracle import OracleTree
from tests.helpers import tie_list

PB_C_BASE, PB_C_INIT, DISC, VDM, NOISE_W = 19652, np.float32(1.25), np.float32(0.997), np.float32(0.01), np.float32(0.25)


def _tree(res, B, A, S, ez):
    ot = OracleTree(B, A, S, ez=ez)
    ot.set_delta(VDM)
    ot.prepare(NOISE_W, res["noises"], np.zeros(B, np.float32), res["logits0"], np.full(B, -1, np.int32))
    return ot


def attribute(ra, rb, B, S, A, ez=False, tau=1e-3):
    """ra / rb: dict(rec=recorder numpy dict with seeds, dist, values, noises, logits0) of two searches"""
    a, b = ra["rec"], rb["rec"]
    assert np.array_equal(a["seeds"], b["seeds"])
    diff_req = (a["x"] != b["x"]) | (a["action"] != b["action"]) | (a["search_len"] != b["search_len"])  # [S, B]
    first = np.where(diff_req.any(axis=0), diff_req.argmax(axis=0), S)
    ta, tb = _tree(ra, B, A, S, ez), _tree(rb, B, A, S, ez)
    rows, gaps = [], []
    vtp0 = np.full(B, -1, np.int32)
    for k in range(S):
        outs = []
        for ot, rec in ((ta, a), (tb, b)):
            x, y, act, vtp, slen = ot.traverse(PB_C_BASE, PB_C_INIT, DISC, int(rec["seeds"][k]), vtp0)
            # the oracle fed this search's own outputs reproduces its GPU tree request for request
            assert np.array_equal(x, rec["x"][k]) and np.array_equal(act, rec["action"][k]) and \
                np.array_equal(slen, rec["search_len"][k]), f"sim {k}: oracle replay differs from the GPU search"
            outs.append((vtp, slen))
        if k % 10 == 0:  # the scale: chosen-vs-runner-up gaps over every level of every walk (search a)
            for i in range(0, B, 8):
                acts = ta.path_actions(i)
                for lvl, sc in enumerate(ta.path_scores(i, acts)):
                    fin = np.sort(sc[np.isfinite(sc)])
                    if len(fin) > 1:
                        gaps.append(float(fin[-1] - fin[-2]))
        for i in np.nonzero(first == k)[0]:
            pa, pb = ta.path_actions(i), tb.path_actions(i)
            lvl = next((l for l in range(min(len(pa), len(pb))) if pa[l] != pb[l]), min(len(pa), len(pb)))
            row = dict(root=int(i), sim=int(k), level=int(lvl), len_a=int(len(pa)), len_b=int(len(pb)))
            if lvl < min(len(pa), len(pb)):
                sa, sb = ta.path_scores(i, pa)[lvl], tb.path_scores(i, pb)[lvl]
                xa, xb = int(pa[lvl]), int(pb[lvl])
                ga, gb = float(abs(sa[xa] - sa[xb])), float(abs(sb[xa] - sb[xb]))
                la, lb = tie_list(sa), tie_list(sb)
                earlier = bool((first[:i] <= k).any())  # a lower root already diverged by this simulation
                if xa in la and xb in la and xa in lb and xb in lb:
                    kind = "draw_shift" if earlier else "tie_draw"
                elif max(ga, gb) <= tau:
                    kind = "near_tie"
                else:
                    kind = "unexplained"
                row.update(action_a=xa, action_b=xb, gap_a=ga, gap_b=gb, kind=kind, lower_root_diverged=earlier,
                           scores_a=[float(v) for v in sa], scores_b=[float(v) for v in sb])
            else:
                row.update(kind="unexplained")
            rows.append(row)
        for ot, rec, (vtp, slen) in ((ta, a, outs[0]), (tb, b, outs[1])):
            is_reset = (slen % 5 == 0).astype(np.int32) if ez else None
            ot.backprop(k + 1, DISC, rec["decoded"][k][:, 0], rec["decoded"][k][:, 1], rec["policy_logits"][k], vtp,
                        is_reset)
    assert np.array_equal(ta.distributions(), ra["dist"]) and np.array_equal(tb.distributions(), rb["dist"])
    differ = (ra["dist"] != rb["dist"]).any(axis=1)
    kinds = {}
    for r in rows:
        kinds[r["kind"]] = kinds.get(r["kind"], 0) + 1
    near = [max(r["gap_a"], r["gap_b"]) for r in rows if r.get("kind") == "near_tie"]
    return dict(B=B, S=S, A=A, roots_visit_counts_differ=int(differ.sum()), rate=float(differ.mean()),
                roots_requests_differ=int((first < S).sum()), first_divergence_kinds=kinds,
                max_near_tie_gap=max(near) if near else None, tau=tau,
                root_value_max_abs_diff_same_counts=float(np.max(np.abs(ra["values"] - rb["values"])[~differ]))
                if (~differ).any() else None,
                # roots whose every request matched (the same tree, only the network's rounding differs)
                root_value_max_abs_diff_same_requests=float(np.max(np.abs(ra["values"] - rb["values"])[first == S]))
                if (first == S).any() else None,
                root_value_max_rel_diff_same_requests=float(np.max(
                    np.abs(ra["values"] - rb["values"])[first == S] / np.maximum(np.abs(ra["values"][first == S]), 1e-6)))
                if (first == S).any() else None,
                typical_gap_quantiles={q: float(np.quantile(gaps, q)) for q in (0.01, 0.1, 0.5)} if gaps else None,
                first_divergences=rows[:64])


def report(name, rep):
    """print the report and write it to $LZM_REPORT_DIR/divergence_<name>.json when set (gpu.sh sets it)"""
    summary = {k: v for k, v in rep.items() if k != "first_divergences"}
    print(f"divergence {name}: {json.dumps(summary)}")
    out = os.environ.get("LZM_REPORT_DIR")
    if out:
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, f"divergence_{name}.json"), "w") as f:
            json.dump(rep, f, indent=1)
