"""Drop-in for the reference's helpers.py (posterior summaries; arviz not needed): epipf.chains_io."""
from epipf.chains_io import gelman_rubin as gelman_rubin_test, hdi, mean_credible_interval, posterior_mse, running_mean  # noqa: F401
