"""Device-resident collect-time search step (first piece).

MuZeroPolicy._forward_collect (lzero/policy/muzero.py:617-690) runs, per env step:
initial_inference -> Roots.prepare (Dirichlet-mixed root priors) -> MuZeroMCTSCtree.search ->
get_distributions / get_values; EfficientZeroPolicy._forward_collect (efficientzero.py:538-656) the
same with the value-prefix roots and the initial inference's reward_hidden_state (LSTM (c, h), zeros)
handed to EfficientZeroMCTSCtree.search. `DeviceSearchStep` runs exactly that sequence on device
tensors — for a MuZero model or, picked from the model (a dynamics network with an LSTM), an
EfficientZero one — and captures it as ONE HIP graph, so a step costs one graph launch: no Python
glue, no host copies between the network, the root preparation and the fused search. The traverse seeds (the
reference's per-call srand(tv_usec) values) are derived on the device from a replay counter,
usec_k = (1000003 * seed + n) mod 10^6 for the n-th traverse of the run (the SequentialSeeds rule
of tests and bench), so every replay is a fresh search.

Inputs are static device buffers the caller refills before `step()` (obs, Dirichlet noises,
to_play) — or that a captured `epilogue` rewrites on the device (the collector's env step);
outputs are static device tensors overwritten by each step (visit counts per legal action, root
values, root latents and policy logits). `step_counter` counts the steps (device int64).
"""
import torch

from .conv_infer import FoldedConvInitial, folded_initial_or_none
from .initial import FusedInitialInference, fused_initial_or_none
from .mcts_ctree import EfficientZeroMCTSCtree, MuZeroMCTSCtree, _step_net
from .utils import EasyDict


class DeviceSearchStep:
    def __init__(self, model, num_envs, num_simulations, legal_actions, obs_shape, device, noise_weight=0.25,
                 discount_factor=0.997, support_scale=300, seed=0, rng_mode="glibc", graph=True, cfg_extra=None,
                 epilogue=None, fused_initial=True):
        self.model = model.eval()
        # initial_inference as one HIP launch when the model is a MuZeroModelMLP (lightzero_amd.initial);
        # for the conv MuZeroModel family its BatchNorm-folded form (conv_infer.FoldedConvInitial)
        self.initial = None
        if fused_initial:
            self.initial = fused_initial_or_none(self.model) or folded_initial_or_none(self.model)
        self._weights_key = None
        self.B, self.S = int(num_envs), int(num_simulations)
        self.device = torch.device(device)
        self.noise_weight = float(noise_weight)
        # EfficientZero models (value prefix + reward LSTM): EfficientZeroMCTSCtree with the policy's
        # lstm_horizon_len (efficientzero.py default 5)
        self.ez = hasattr(getattr(model, "dynamics_network", None), "lstm")
        cfg = dict(num_simulations=self.S, discount_factor=float(discount_factor), device=self.device,
                   model=dict(support_scale=int(support_scale), categorical_distribution=True))
        if self.ez:
            cfg["lstm_horizon_len"] = 5
        cfg.update(cfg_extra or {})
        self.mcts_cls = EfficientZeroMCTSCtree if self.ez else MuZeroMCTSCtree
        self.rng_mode = rng_mode
        self.mcts = self.mcts_cls(EasyDict(cfg))
        self.legal = [list(l) for l in legal_actions]
        self.A = max(len(l) for l in self.legal)
        dev = self.device
        self.obs = torch.zeros((self.B,) + tuple(obs_shape), dtype=torch.float32, device=dev)
        self.noises = torch.zeros((self.B, self.A), dtype=torch.float32, device=dev)
        self.to_play = torch.full((self.B,), -1, dtype=torch.int32, device=dev)
        self.rewards = torch.zeros(self.B, dtype=torch.float32, device=dev)
        self._count = torch.zeros(1, dtype=torch.int64, device=dev)
        self._base = (1000003 * int(seed)) % 1000000
        self._ar = torch.arange(self.S, dtype=torch.int64, device=dev)
        self.graph = None
        self.use_graph = bool(graph)
        self.epilogue = epilogue  # fn(out dict), enqueued after the search inside the same graph
        self.roots = None
        self.out = None

    def set_inputs(self, obs=None, noises=None, to_play=None):
        if obs is not None:
            self.obs.copy_(obs)
        if noises is not None:
            self.noises.copy_(noises)
        if to_play is not None:
            self.to_play.copy_(to_play)

    def _body(self):
        with torch.no_grad():
            old = self.mcts_cls.rng_mode
            self.mcts_cls.rng_mode = self.rng_mode
            try:
                if self.roots is None:
                    self.roots = self.mcts_cls.roots(self.B, self.legal)
                pool0 = self._root_slot() if isinstance(self.initial, FusedInitialInference) else None
                if pool0 is not None:
                    # one launch: initial_inference into the search's root slot (the search skips its
                    # copy) and the root preparation from the policy logits
                    out = self.initial.initial_inference(
                        self.obs, latent_out=pool0,
                        prepare=dict(roots=self.roots, noise_weight=self.noise_weight, noises=self.noises,
                                     rewards=self.rewards, to_play=self.to_play))
                else:
                    prepared = False
                    if isinstance(self.initial, FoldedConvInitial):
                        # the latent straight into the root slot; the root preparation in the heads' launch
                        out = self.initial.initial_inference(
                            self.obs, latent_out=self._root_slot(),
                            prepare=dict(roots=self.roots, noise_weight=self.noise_weight, noises=self.noises,
                                         rewards=self.rewards, to_play=self.to_play))
                        prepared = getattr(out, "prepared", False)
                    else:
                        out = (self.initial or self.model).initial_inference(self.obs)
                    if not prepared:
                        self.roots.prepare_device(self.noise_weight, self.noises, self.rewards, out.policy_logits,
                                                  self.to_play)
                # the seeds (from the step counter), fresh min-max bounds, the root outputs and the
                # counter increment run inside the search (the one-launch search: in its kernel); an
                # epilogue (the collector's env step) reads the advanced counter
                t = self.roots.tree
                dist = torch.empty((self.B, t.A), dtype=torch.int32, device=self.device)
                values = torch.empty(self.B, dtype=torch.float32, device=self.device)
                stp = dict(count=self._count, base=self._base, dist=dist, values=values, increment=True)
                if self.ez:  # the roots' LSTM state: the initial inference's reward_hidden_state (zeros)
                    self.mcts.search(self.roots, self.model, out.latent_state, out.reward_hidden_state, self.to_play,
                                     step=stp)
                else:
                    self.mcts.search(self.roots, self.model, out.latent_state, self.to_play, step=stp)
                res = dict(distributions=dist, values=values, latent_state=out.latent_state,
                           policy_logits=out.policy_logits, value_logits=out.value)
                if self.epilogue is not None:
                    self.epilogue(res)
                return res
            finally:
                self.mcts_cls.rng_mode = old

    def _root_slot(self):
        """the search's root latent slot (pool[0]) once its buffers exist, else None"""
        buf = getattr(self.mcts, "_buf", None)
        pool = getattr(buf, "pool", None) if buf is not None and buf.key is not None else None
        return pool[0] if pool is not None and pool.shape[1] == self.B else None

    def build_graph(self):
        """Warm up (allocations: tree handle, glibc tables, packed weights, torch workspaces) and
        capture the body; runs the body twice eagerly, so callers with device state re-initialise it
        afterwards. The step counter restarts at 0."""
        if not self.use_graph or self.graph is not None:
            return
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(2):
                self._body()
        torch.cuda.current_stream(self.device).wait_stream(s)
        self._count.zero_()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.out = self._body()

    def _weights_version(self):
        m = self.model
        return tuple(x._version for x in list(m.parameters()) + list(m.buffers()))

    def refresh_weights(self):
        """Re-pack the network for the captured kernels if its parameters changed (e.g. a learner
        update): both caches re-pack IN PLACE, so the captured graph reads the new weights. A graph
        replay runs no Python, so this host-side version check runs before every replay: one cached
        tuple compare of the model's tensor versions, the caches only when it changed."""
        key = self._weights_version()
        if key == self._weights_key:
            return
        self._weights_key = key
        if self.initial is not None:
            self.initial.refresh()
        if self.roots is not None and self.roots.tree is not None:
            fused = getattr(self.mcts, "_fused", None)  # (MuZero's packed-MLP one-launch search)
            if fused is None or fused(self.model, self.roots.tree) is None:
                # conv models (MuZero or EfficientZero): the folded step network re-folds in place
                _step_net(self.mcts, self.model)

    def step(self):
        """One collect-time search pass over the current inputs; returns the static output dict."""
        if not self.use_graph:
            self.out = self._body()
            return self.out
        self.build_graph()
        self.refresh_weights()
        self.graph.replay()
        if self.roots is not None and self.roots.tree is not None:
            self.roots.tree.searched()
        return self.out

    def reset_seed_counter(self):
        self._count.zero_()

    @property
    def step_counter(self):
        return self._count
