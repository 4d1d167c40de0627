"""epipf: MI355X-native bootstrap particle filter / PMCMC for stochastic epidemic models.

Drop-in for the reference's pmcmc.py hot path (particle_filter, particle_path_sampler,
particle_mcmc, ModelType) and its Gillespie simulators, with the filter running as HIP kernels in
libepipf.so (C ABI: include/epipf.h).  See DESIGN.md.
"""
from .engine import Engine, get_engine  # noqa: F401
from .pmcmc import (ModelType, chain_key, particle_filter, particle_mcmc, particle_mcmc_chains,  # noqa: F401
                    particle_path_sampler, seed_stream)
from .gillespie import (sir_simulate, seir_simulate, sir_subgroups_simulate, simulate_batch,  # noqa: F401
                        simulate_path_batch)
from .abc import abc_algo, abc_run  # noqa: F401

__all__ = ["Engine", "get_engine", "ModelType", "particle_filter", "particle_mcmc", "particle_mcmc_chains",
           "particle_path_sampler", "seed_stream", "chain_key", "sir_simulate", "seir_simulate",
           "sir_subgroups_simulate", "simulate_batch", "simulate_path_batch", "abc_algo", "abc_run"]
