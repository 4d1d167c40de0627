"""Test double for epipf.engine.Engine that answers from the CPU oracle (TEST INFRASTRUCTURE ONLY).

Used by the CPU tests of the host logic (MH loop, multi-chain lockstep, distributed sharding) so they run
without a GPU.  The product has no such fallback: epipf.engine.Engine always requires libepipf.so + a GPU."""
import numpy as np

import oracle
from epipf.engine import model_id, n_compartments


class OracleEngine:
    """Test double with Engine's interface (set_observations / set_population / run / path_sample)."""

    def __init__(self, mid, G, N, T, chains):
        self.mid, self.G, self.N, self.t_max, self.max_chains = mid, G, N, T, chains
        self.model = mid
        self.C = n_compartments(mid, G)
        self.hist = {}

    def set_observations(self, Y):
        self.Y = np.asarray(Y, dtype=float)
        self.T = self.Y.shape[0]

    def set_population(self, npop, mu):
        self.npop, self.mu = np.atleast_1d(npop), np.atleast_1d(mu)

    def run(self, thetas, probs, keys, fidx, observations=False, active=None, resample="multinomial", chosen=None):
        n = len(thetas)
        probs = np.broadcast_to(probs, (n,))
        keys = np.broadcast_to(np.asarray(keys, dtype=np.uint64), (n,))
        fidx = np.broadcast_to(fidx, (n,))
        lz = np.zeros((n, self.T))
        st = np.zeros(n, dtype=np.int32)
        name = ["sir", "seir", "sir_subgroups", "sir_subgroups2"][self.mid]
        for c in range(n):
            if active is not None and not active[c]:
                st[c] = 2
                continue
            th = thetas[c]
            if self.mid >= 2:
                th = (th[:self.G * self.G].reshape(self.G, self.G), th[-1])
            npop = self.npop if self.mid >= 2 else float(self.npop[0])
            mu = self.mu if self.mid >= 2 else float(self.mu[0])
            o = oracle.particle_filter(self.Y, name, th, observations, float(probs[c]), self.N, npop, mu,
                                       key=int(keys[c]), filter_index=int(fidx[c]), resample=resample)
            st[c] = o["status"]
            lz[c] = o["log_zetas"]
            self.hist[c] = (o["hidden"], o["ancestry"])
        if chosen is None:
            return lz, st
        # epipf_run_sampled: the path sampler on the picks handed over with the filter (zeros: -1 or not OK)
        tr = np.zeros((n, self.T, self.C), dtype=np.int32)
        for c in range(n):
            if st[c] == 0 and chosen[c] >= 0:
                tr[c] = self._walk(c, int(chosen[c]))
        return lz, st, tr

    def _walk(self, c, ch):
        hid, anc = self.hist[c]
        out = np.zeros((self.T, self.C), dtype=np.int32)
        out[-1] = hid[-1, ch]
        for p in range(self.T - 2, -1, -1):
            ch = anc[p, ch]
            out[p] = hid[p, ch]
        return out

    def path_sample(self, chosen):
        out = np.zeros((len(chosen), self.T, self.C), dtype=np.int32)
        for c, ch in enumerate(chosen):
            if c in self.hist:
                out[c] = self._walk(c, int(ch))
        return out


def fake_get_engine(type_model, groups, n_particles, T, chains=1, device=0):
    mid = model_id(type_model)
    return OracleEngine(mid, groups if mid >= 2 else 1, int(n_particles), T, chains)
