"""Generates tests/golden/az_*.npz from the REFERENCE AlphaZero tree (oracle/_ref/mcts_alphazero,
built by oracle/build_ref.sh from lzero/mcts/ctree/ctree_alphazero/mcts_alphazero.cpp) driven with the
restated TicTacToe simulate-env and the scripted float-exact policy-value function
(oracle/tictactoe.py). Run in the build container: python tests/golden/gen_golden_az.py

Each case stores the boards, start players, num_simulations, whether root noise was added
(sample=True: the reference's default-seeded gamma noise) and the returned action_probs (root
visit counts / num_simulations at temperature 1). The final sampled action uses std::random_device
in the reference and is not recorded.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle", "_ref"))

import mcts_alphazero  # noqa: E402  (the reference, compiled here)

from oracle.tictactoe import SimTicTacToe, random_boards, scripted_policy_value  # noqa: E402

CASES = [  # name, n boards, sims, sample (root noise), seed
    ("az_s25_nonoise", 48, 25, False, 1),
    ("az_s100_nonoise", 32, 100, False, 2),
    ("az_s50_noise", 48, 50, True, 3),
    ("az_s200_noise", 16, 200, True, 4),
]


def run_case(n, sims, sample, seed):
    boards, starts = random_boards(n, seed)
    env = SimTicTacToe(scale=True)
    mcts = mcts_alphazero.MCTS(9, sims, 19652, 1.25, 0.3, 0.25, env)

    def pv(e):
        return scripted_policy_value(e.board.reshape(-1), e.legal_actions)

    probs = []
    for b, s in zip(boards, starts):
        cfg = dict(start_player_index=int(s), init_state=b.reshape(3, 3).astype(np.int32), katago_policy_init=False,
                   katago_game_state=None)
        _, p = mcts.get_next_action(cfg, pv, 1.0, bool(sample))
        probs.append(p)
    return boards, starts, np.array(probs, np.float64)


def main():
    for name, n, sims, sample, seed in CASES:
        boards, starts, probs = run_case(n, sims, sample, seed)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), boards=boards, starts=starts, sims=sims,
                            sample=sample, action_probs=probs)
        print(name, boards.shape, probs.shape)


if __name__ == "__main__":
    main()
