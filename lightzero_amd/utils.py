"""Small host utilities shared by the drop-in classes."""
try:  # the reference uses easydict.EasyDict for every config (mcts_ctree.py:7)
    from easydict import EasyDict  # type: ignore
except ImportError:  # not installed in this image: equivalent attribute dict
    class EasyDict(dict):
        """dict with attribute access; nested dicts become EasyDicts (easydict semantics)."""

        def __init__(self, d=None, **kw):
            super().__init__()
            d = dict(d or {}, **kw)
            for k, v in d.items():
                self[k] = v

        def __setitem__(self, k, v):
            if isinstance(v, dict) and not isinstance(v, EasyDict):
                v = EasyDict(v)
            elif isinstance(v, (list, tuple)):
                v = type(v)(EasyDict(x) if isinstance(x, dict) and not isinstance(x, EasyDict) else x for x in v)
            super().__setitem__(k, v)

        __setattr__ = __setitem__

        def __getattr__(self, k):
            try:
                return self[k]
            except KeyError as e:
                raise AttributeError(k) from e

        def __delattr__(self, k):
            del self[k]

        def update(self, e=None, **f):
            d = dict(e or {}, **f)
            for k, v in d.items():
                self[k] = v

        def __deepcopy__(self, memo):
            import copy
            return EasyDict({k: copy.deepcopy(v, memo) for k, v in self.items()})
