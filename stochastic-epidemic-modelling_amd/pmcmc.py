"""Drop-in module: `sys.path.append('<repo>/stochastic-epidemic-modelling_amd'); from pmcmc import *`
gives the reference's pmcmc.py names (ModelType, particle_filter, particle_path_sampler,
particle_mcmc, *_simulate_discrete returning the reference's DataFrames, the differential_* right-hand sides
including the reference's `differential_sir_subroups` spelling) backed by the MI355X engine."""
from epipf.pmcmc import (ModelType, particle_filter, particle_mcmc, particle_mcmc_chains,  # noqa: F401
                         particle_path_sampler, seed_stream)
from epipf.datasets import (differential_seir, differential_sir, differential_sir_subgroups,  # noqa: F401
                            differential_sir_subroups, seir_simulate_discrete, sir_simulate_discrete,
                            sir_subgroups_simulate_discrete)
from epipf.gillespie import seir_simulate, sir_simulate, sir_subgroups_simulate  # noqa: F401
