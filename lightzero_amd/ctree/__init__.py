"""GPU-backed replacements of LightZero's Cython ctree modules (mz_tree, ez_tree)."""
