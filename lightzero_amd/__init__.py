"""lightzero_amd — MI355X-native batched MuZero / EfficientZero MCTS (drop-in for LightZero's
ctree search path). See DESIGN.md. Requires the in-tree liblzmcts.so (built for gfx950)."""
from . import _lib  # noqa: F401

__version__ = "0.1.0"


def __getattr__(name):
    # lazy: importing the package must not touch the GPU
    if name in ("MuZeroMCTSCtree", "EfficientZeroMCTSCtree"):
        from . import mcts_ctree
        return getattr(mcts_ctree, name)
    if name == "InverseScalarTransform":
        from .scaling_transform import InverseScalarTransform
        return InverseScalarTransform
    raise AttributeError(name)
