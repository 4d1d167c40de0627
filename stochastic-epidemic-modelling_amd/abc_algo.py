"""Drop-in module mirroring the reference's abc_algo.py names (the rejection loop runs on the GPU)."""
from epipf.abc import abc_algo, abc_run, distance_function  # noqa: F401
