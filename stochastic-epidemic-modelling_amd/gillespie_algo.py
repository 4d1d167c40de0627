"""Drop-in module mirroring the reference's gillespie_algo.py names (last-value and full-path modes on the GPU)."""
from epipf.gillespie import (seir_simulate, simulate_batch, simulate_path_batch, sir_simulate,  # noqa: F401
                             sir_subgroups_simulate)
