"""Drop-in module mirroring the reference's gillespie_algo.py names (last_values_only=True on the GPU)."""
from epipf.gillespie import seir_simulate, simulate_batch, sir_simulate, sir_subgroups_simulate  # noqa: F401
