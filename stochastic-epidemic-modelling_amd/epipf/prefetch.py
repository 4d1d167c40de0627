"""Prefetching (speculative) Metropolis-Hastings: one PMCMC chain advanced several iterations per GPU batch.

The reference's MH loop (pmcmc.py:325-406) runs one particle filter per iteration, and iteration i+1's
proposal depends on whether iteration i accepted, so a single chain is a sequential chain of filters.  One
filter of N = 10^4 particles fills ~160 of the GPU's 1024 SIMDs; a single chain therefore runs at a small
fraction of what the chip can do.  Prefetching MCMC (Brockwell 2006; Strid 2010) evaluates the filters of
several FUTURE iterations at once, one per node of the tree of accept/reject outcomes:

  * every random number the MH loop draws on the host (the proposal's standard normals, the path sampler's
    randint, the acceptance uniform) comes from the chain's RandomState in a fixed per-iteration pattern that
    does not depend on accept/reject: an iteration consumes d normals, then a pick and a uniform if its filter
    ran and succeeded.  So every node at the same depth of the tree reads the same position of ONE replayed
    stream (a clone of the RandomState drawn ahead once), and the proposal is numpy's legacy
    multivariate_normal arithmetic on those normals: x = z @ (sqrt(s) v), x += mean (bit-identical, checked);
    a negative proposal or a degenerate filter consumes the normals only, and its subtree forks a new stream
    (rare: a replay from the stream's start).  The caller's RandomState advances along the realised path with
    the same calls, so it ends exactly where the sequential loop leaves it;
  * every filter is a pure function of (theta, probs, Philox key, filter index), and a node's
    filter index is the count of filters on its path, so a speculative filter returns exactly what the
    sequential run's filter would;
  * each round schedules the K most probable unevaluated nodes (best first: accept branch weighted by the
    chain's observed acceptance rate), runs their filters as ONE batched launch sequence (epipf_run over K
    chain slots) plus on-device path sampling, then walks the realised path from the root as far as results
    reach.  Nodes off the realised path are discarded; evaluated nodes below the new root are kept.

The committed thetas, likelihoods, trajectories, acceptance count, filter count and the final RandomState
state are identical to `ChainSampler`'s sequential run (tests/test_prefetch.py, tests/test_gpu_parity.py).
"""
import heapq
import itertools

import numpy as np

from . import _lib
from .pmcmc import ChainSampler, _log_ratio, _reference_ratio, mvn_apply, mvn_factor


class _Val:
    """A committed likelihood / trajectory (the root's current state)."""
    __slots__ = ("z", "lz", "traj")

    def __init__(self, z, lz, traj):
        self.z, self.lz, self.traj = z, lz, traj


class _Stream:
    """A clone of a chain's RandomState drawn ahead in the standard per-iteration pattern: position k holds the
    proposal normals z (pmcmc.py:330), the path pick (:241) and the acceptance uniform (:395) of the k-th
    iteration after the stream's start."""
    SNAP = 32                       # a state snapshot every SNAP positions bounds a fork's replay

    __slots__ = ("snaps", "rs", "z", "chosen", "u", "forks", "d", "N")

    def __init__(self, state, d, N):
        self.rs = np.random.RandomState()
        self.rs.set_state(state)
        self.snaps = {0: state}
        self.z, self.chosen, self.u, self.forks = [], [], [], {}
        self.d, self.N = d, N

    def at(self, k):
        while len(self.z) <= k:
            n = len(self.z)
            if n % self.SNAP == 0 and n not in self.snaps:
                self.snaps[n] = self.rs.get_state()
            self.z.append(self.rs.standard_normal(self.d))
            self.chosen.append(self.rs.randint(0, self.N))
            self.u.append(self.rs.random_sample())           # == uniform() (0 + 1*U), same draw
        return self.z[k], self.chosen[k], self.u[k]

    def fork(self, k):
        """The stream after k standard iterations and the normals of one more (a negative proposal, or a filter
        that returned (None, None, None): no pick and no uniform drawn)."""
        f = self.forks.get(k)
        if f is None:
            self.at(k)
            k0 = (k // self.SNAP) * self.SNAP
            rs = np.random.RandomState()
            rs.set_state(self.snaps[k0])
            for _ in range(k - k0):
                rs.standard_normal(self.d)
                rs.randint(0, self.N)
                rs.random_sample()
            rs.standard_normal(self.d)
            f = self.forks[k] = _Stream(rs.get_state(), self.d, self.N)
        return f


class _DegRef:
    """A degenerate-filter child in the scheduler's heap, created (a stream fork: RandomState replay) only once popped."""
    __slots__ = ("x",)

    def __init__(self, x):
        self.x = x


class _Node:
    """State before MH iteration `i` on one path of one chain's outcome tree."""
    __slots__ = ("chain", "i", "parent", "theta", "src", "stream", "k", "fnext", "chosen", "u", "prop", "neg",
                 "stripped", "theta_new", "result", "kids", "deg")

    def __init__(self, chain, i, parent, theta, src, stream, k, fnext):
        self.chain, self.i, self.parent = chain, i, parent
        self.theta = theta          # theta_{i-1}: the proposal mean
        self.src = src              # _Val, or the filter node whose result is this state's likelihood
        self.stream, self.k = stream, k   # host draws of iteration i: position k of the stream
        self.fnext = fnext          # filter index of the next filter on this path
        self.chosen = self.u = None
        self.prop = None
        self.neg = False
        self.stripped = None
        self.theta_new = None
        self.result = None          # (log_zetas [T], status, trajectory [T, C]) once the filter ran
        self.kids = None            # (accept, reject) or (negative,)
        self.deg = None


def _value(src):
    """(z, lz, traj) of a node's current state, or None while its filter has not run."""
    if isinstance(src, _Val):
        return src.z, src.lz, src.traj
    if src.result is None:
        return None
    lz = src.result[0]
    return np.exp(lz[-1]), lz[-1], src.result[2]


def expected_iterations_upto(kmax, alphas, deltas=None):
    """[E(1), ..., E(kmax)] of expected_iterations from one best-first expansion (the scheduled nodes of K slots are
    the first K of K + 1's)."""
    deltas = [0.0] * len(alphas) if deltas is None else deltas
    heap = [(-1.0, c) for c in range(len(alphas))]
    heapq.heapify(heap)
    e, out = 0.0, []
    for _ in range(int(kmax)):
        if heap:
            negp, c = heapq.heappop(heap)
            e -= negp
            a, d = alphas[c], deltas[c]
            heapq.heappush(heap, (negp * (1.0 - d) * a, c))
            heapq.heappush(heap, (negp * (1.0 - d) * (1.0 - a), c))
            if d > 0.0:
                heapq.heappush(heap, (negp * d, c))
        out.append(e)
    return out


def expected_iterations(slots, alphas, deltas=None):
    """Expected MH iterations one round commits when `slots` filters are scheduled best-first over chains whose
    accept probability is `alphas` and whose filters degenerate with probability `deltas` (the scheduler of
    PrefetchSampler._schedule on the ideal tree: every node a filter with three outcomes -- degenerate (d), accepted
    ((1 - d) a), rejected ((1 - d)(1 - a)) -- path probability = product along it; a round commits the realised path's
    evaluated prefix, so the expectation is the sum of the scheduled nodes' path probabilities)."""
    deltas = [0.0] * len(alphas) if deltas is None else deltas
    heap = [(-1.0, c) for c in range(len(alphas))]
    heapq.heapify(heap)
    e = 0.0
    for _ in range(int(slots)):
        if not heap:
            break
        negp, c = heapq.heappop(heap)
        e -= negp
        a, d = alphas[c], deltas[c]
        heapq.heappush(heap, (negp * (1.0 - d) * a, c))
        heapq.heappush(heap, (negp * (1.0 - d) * (1.0 - a), c))
        if d > 0.0:
            heapq.heappush(heap, (negp * d, c))
    return e


class SlotTuner:
    """slots="auto": the round width that maximises committed filters per second of wall time.  A round's
    wall time T(K) grows with its K filters once they no longer fit the idle SIMDs (the lane-group kernel and
    the chip's fill set where), and its yield E(K) grows sub-linearly at a rate set by the acceptance rate, so the best
    K depends on both.  T(K) is measured on the chain's own rounds -- each candidate power of two run once to warm up
    (not timed: a first launch shape pays one-off costs) and then `tries` times, T(K) the median of its last five rounds
    (a round lasts as long as its slowest filter, and the filters' costs vary with their theta: at config 5's h = 1 a
    fastest-of-three estimate picked 4 slots in one run and 1 in another, profiles/r4y_prefetch_cfg5.txt); the best and
    its neighbours re-measured every `refresh` rounds, an interval that doubles (up to `refresh_max`) each time the
    re-measurement leaves the best width where it was and starts again at `refresh` when it moves it (a refresh round
    at twice the width costs about two rounds: at a fixed interval of 24 it cost config 2 ~5-9%, BENCH_r05).
    E(K) is OBSERVED, not modelled: the scheduler is best-first, so the K' < K most probable nodes of a K-slot round are
    exactly what a K'-slot round would have run from the same root, and a round at width K therefore also tells what
    every narrower width would have committed (PrefetchSampler._resolve: the realised path cut at its first node of
    schedule rank >= K').  Every round adds one sample to each width up to its own; the tree model
    (expected_iterations, independent accept / reject at the running rates) only seeds the estimate while samples are
    few (weight `prior` rounds) -- on its own it overstated wide rounds (config 2, acceptance 0.08: E(32) / E(16) = 1.28
    modelled, 1.07 observed, so 32 slots were picked and ran 10% slower than 16, BENCH_r04)."""

    def __init__(self, lo, hi, tries=3, refresh=24, reeval=8, prior=2, window=64, refresh_max=384):
        self.cands = sorted({lo} | {k for k in (1, 2, 4, 8, 16, 32, 64, 128) if lo <= k <= hi} | {hi})
        self.samples = {k: [] for k in self.cands}          # K -> the last round times (s)
        self.count = {k: 0 for k in self.cands}              # rounds run at K (the first is a warm-up)
        self.yields = {k: [] for k in self.cands}           # K -> filters a K-slot round committed (observed or
                                                             # cut from a wider round), the last `window`
        self.tries, self.refresh, self.reeval, self.prior, self.window = tries, refresh, reeval, prior, window
        self.rounds = 0
        self.best = None
        self._next_eval = 0
        self.refresh0, self.refresh_max = refresh, refresh_max
        self._next_refresh = None                            # round of the next neighbour re-measurement
        self._refreshes = 0

    def time(self, k):
        return float(np.median(self.samples[k][-5:]))

    def pick(self, alphas, deltas=None):
        for k in self.cands:                                # exploration: every candidate measured `tries` times
            if len(self.samples[k]) < self.tries:
                return k
        # the argmax moves only with new round times or acceptance estimates: re-evaluated every `reeval` rounds (one
        # heap expansion for every width; per round it cost ~5% of a 2-slot config-5 round in Python)
        if self.best is None or self.rounds >= self._next_eval:
            E = expected_iterations_upto(self.cands[-1], alphas, deltas)
            best = max(self.cands, key=lambda k: self.yield_of(k, E[k - 1]) / self.time(k))
            if self.best is not None and best != self.best:  # the width moved: re-measure its neighbours often again
                self.refresh = self.refresh0
            self.best = best
            self._next_eval = self.rounds + self.reeval
        if self._next_refresh is None:
            self._next_refresh = self.rounds + self.refresh
        if self.rounds >= self._next_refresh:               # keep the neighbours' times current, alternately
            self._refreshes += 1
            self._next_refresh = self.rounds + self.refresh
            if self._refreshes % 2 == 0:                    # both neighbours seen since the last change: back off
                self.refresh = min(self.refresh_max, 2 * self.refresh)
            i = self.cands.index(self.best)
            j = i - 1 if self._refreshes % 2 == 1 else i + 1
            if not 0 <= j < len(self.cands):
                j = i + 1 if j < i else i - 1
            if 0 <= j < len(self.cands):
                return self.cands[j]
        return self.best

    def yield_of(self, k, model):
        """Filters a round of K commits: the mean of the observed yields of width K (its own rounds and the cuts of
        wider ones), the tree model's E(K) counting as `prior` rounds."""
        obs = self.yields[k]
        return (sum(obs) + self.prior * model) / (len(obs) + self.prior)

    def record(self, k, seconds, committed=None):
        """A round of width k took `seconds`; committed: {K': filters a K'-slot round would have committed} for the
        candidates K' <= k (PrefetchSampler._resolve), or the round's own count."""
        self.rounds += 1
        if committed is not None:
            cuts = committed if isinstance(committed, dict) else {k: committed}
            for kk, v in cuts.items():
                if kk in self.yields:
                    self.yields[kk] = (self.yields[kk] + [v])[-self.window:]
        if k not in self.count:
            return
        self.count[k] += 1
        if self.count[k] > 1:
            self.samples[k] = (self.samples[k] + [seconds])[-5:]


class PrefetchSampler(ChainSampler):
    """`ChainSampler` (same arguments, same results) that evaluates up to `slots` speculative MH iterations per
    batched filter launch, shared best-first among its chains.  slots="auto" sizes each round from the observed
    acceptance rate and the measured round time (SlotTuner); results do not depend on the width."""

    def __init__(self, *args, slots=32, **kw):
        n_particles = args[9] if len(args) > 9 else kw.get("n_particles", 1000)
        n_chains = len(kw["rngs"]) if "rngs" in kw else 1
        self.tuner = None
        if slots == "auto":
            from .pmcmc import prefetch_slots
            hi = max(n_chains, min(64, 2 * prefetch_slots(n_particles)))
            self.tuner = SlotTuner(max(1, n_chains), hi)
            slots = hi
        self.slots = max(1, int(slots))
        kw["engine_chains"] = max(self.slots, int(kw.get("engine_chains", 0)))
        super().__init__(*args, **kw)
        self._std0 = [s.copy() for s in self.std]
        self._factor0 = [self._factor(s) for s in self._std0]
        self.roots = None
        self._tick = itertools.count()
        self.rounds = 0
        self.speculative_filters = 0
        self.degenerate = 0                                     # realised filters that returned (None, None, None)
        self.degenerate_c = [0] * self.nc                       # the same per chain (the scheduler's third branch)
        self._rank = {}

    # ------------------------------------------------------------------ host draws
    def _factor(self, std):
        """sqrt(s)[:, None] * vh of svd(h * std): numpy's legacy multivariate_normal transform."""
        return mvn_factor(self.h * std)

    def _std_for(self, node):
        """Proposal covariance factor at iteration node.i (pmcmc.py:326-328: adaptive after 1000 iterations)."""
        if not (self.adaptive and node.i > 1e3):
            return self._std0[node.chain]
        path = []
        n = node
        while n is not self.roots[node.chain]:
            path.append(n.theta)
            n = n.parent
        th = np.concatenate([self.thetas[node.chain, :n.i], np.array(path[::-1]).reshape(-1, self.d)], axis=0)
        return np.cov(th[:node.i].T, ddof=0) + 1e-4 * np.eye(self.d)

    def _expand(self, x):
        """Proposal of iteration x.i and x's children (accept / reject, or the negative-proposal pass)."""
        if x.kids is not None:
            return
        z, x.chosen, x.u = x.stream.at(x.k)
        if self.adaptive and x.i > 1e3:
            fac = self._factor(self._std_for(x))
        else:
            fac = self._factor0[x.chain]
        prop = mvn_apply(z, fac, x.theta)                       # == multivariate_normal(theta, h*std), pmcmc.py:330
        x.prop = prop
        if (prop < 0).any():                                    # sum(prop < 0) > 0, pmcmc.py:333-337: no filter
            x.neg = True
            x.kids = (_Node(x.chain, x.i + 1, x, x.theta, x.src, x.stream.fork(x.k), 0, x.fnext),)
            return
        th, p2 = self._split(prop)
        x.stripped = (th, p2)
        x.theta_new = np.append(th, p2) if self.probs is None else prop
        x.kids = (_Node(x.chain, x.i + 1, x, x.theta_new, x, x.stream, x.k + 1, x.fnext + 1),
                  _Node(x.chain, x.i + 1, x, x.theta, x.src, x.stream, x.k + 1, x.fnext + 1))

    def _degenerate_child(self, x):
        if x.deg is None:                                       # pmcmc.py:365-369: no pick, no uniform drawn
            x.deg = _Node(x.chain, x.i + 1, x, x.theta, x.src, x.stream.fork(x.k), 0, x.fnext + 1)
        return x.deg

    def _decision(self, x):
        """Realised child of an evaluated node, or None while its current likelihood is unknown."""
        lzr, status, _ = x.result
        if status != _lib.STATUS_OK:
            return self._degenerate_child(x)
        cur = _value(x.src)
        if cur is None:
            return None
        z_old, lz_old, _ = cur
        z_new = np.exp(lzr[-1])
        if self.mh_ratio == "reference":
            prob = _reference_ratio(z_new, z_old, x.theta_new, x.theta, self.params[x.chain], self.h * self._std_for(x))
        else:
            prob = _log_ratio(lzr[-1], lz_old)
        return x.kids[0] if x.u < prob else x.kids[1]

    # ------------------------------------------------------------------ rounds
    def _alpha(self, c):
        """Accept probability of a chain's filter that did not degenerate."""
        ok = self.filters_run[c] - self.degenerate_c[c]
        return (self.acceptances[c] - 1 + 1.0) / (ok + 2.0)

    def _delta(self, c):
        """Probability that a chain's filter degenerates (all weights 0: pmcmc.py:187-192), the realised rate.  At
        config 5's h = 1 about a fifth of the filters do (profiles/r4v_chain_cost_cfg5.txt), and their subtree forks
        the RNG stream (no path pick, no acceptance uniform), so a tree of accept / reject branches alone commits
        about 1 / 0.2 iterations per round whatever its width."""
        return self.degenerate_c[c] / (self.filters_run[c] + 2.0)

    def _push_children(self, heap, x, p):
        """The unevaluated filter node x's three outcomes, best-first by path probability."""
        a, d = self._alpha(x.chain), self._delta(x.chain)
        heapq.heappush(heap, (-p * (1.0 - d) * a, next(self._tick), x.kids[0]))
        heapq.heappush(heap, (-p * (1.0 - d) * (1.0 - a), next(self._tick), x.kids[1]))
        if d > 0.0:
            heapq.heappush(heap, (-p * d, next(self._tick), _DegRef(x)))

    def _schedule(self):
        heap = []
        for c, r in enumerate(self.roots):
            heapq.heappush(heap, (-1.0, next(self._tick), r))
        out = []
        while heap and len(out) < self.slots:
            negp, _, x = heapq.heappop(heap)
            p = -negp
            if isinstance(x, _DegRef):
                x = self._degenerate_child(x.x)
            if x.i >= self.iters:
                continue
            self._expand(x)
            if x.neg:
                heapq.heappush(heap, (-p, next(self._tick), x.kids[0]))
                continue
            if x.result is None:
                out.append(x)
                self._push_children(heap, x, p)
                continue
            y = self._decision(x)
            if y is not None:
                heapq.heappush(heap, (-p, next(self._tick), y))
            else:                                               # its filter ran and did not degenerate
                a = self._alpha(x.chain)
                heapq.heappush(heap, (-p * a, next(self._tick), x.kids[0]))
                heapq.heappush(heap, (-p * (1.0 - a), next(self._tick), x.kids[1]))
        return out

    def _evaluate(self, nodes):
        n = len(nodes)
        th_all = np.zeros((n, self.dth))
        pr_all = np.zeros(n)
        keys = np.zeros(n, dtype=np.uint64)
        fidx = np.zeros(n, dtype=np.uint64)
        for s, x in enumerate(nodes):
            th_all[s], pr_all[s] = x.stripped
            keys[s] = self.keys[x.chain]
            fidx[s] = x.fnext
        self._bind()
        lz, st = self.eng.run(th_all, pr_all, keys, fidx, observations=self.observations, resample=self.resample)
        chosen = np.array([x.chosen for x in nodes], dtype=np.int32)
        tr = self.eng.path_sample(chosen) if np.any(st == _lib.STATUS_OK) else None
        for s, x in enumerate(nodes):
            x.result = (lz[s].copy(), int(st[s]), None if tr is None else tr[s])
        self._rank = {id(x): s for s, x in enumerate(nodes)}    # this round's schedule ranks (best-first order)
        self.last_active = n
        self.speculative_filters += n
        self.rounds += 1

    def _commit(self, c, x, y, filtered, accepted):
        """Iteration x.i realised as y.  The caller's RandomState draws what the sequential loop would."""
        rng = self.rngs[c]
        rng.standard_normal(self.d)                             # the proposal's normals (multivariate_normal)
        if filtered and x.result[1] == _lib.STATUS_OK:
            rng.randint(0, self.N)                              # path pick, pmcmc.py:241
            rng.random_sample()                                 # acceptance uniform (== uniform()), :395
        i = x.i
        z, lz, traj = _value(y.src)
        self.thetas[c, i] = y.theta
        self.likelihoods[c, i] = z
        self.loglik[c, i] = lz
        self.trajs[c, :, i, :] = traj
        if filtered:
            self.filters_run[c] += 1
        if accepted:
            self.acceptances[c] += 1

    def _resolve(self, widths=()):
        """Walk every chain's realised path as far as the evaluated filters reach; returns (iterations committed,
        {K': realised-path filters a K'-slot round would have committed} for K' in widths).  The cut for K' ends each
        chain's walk at its first filter of this round's schedule rank >= K' (best-first: a K'-slot round runs the same
        first K' nodes)."""
        done = 0
        cut = dict.fromkeys(widths, 0)
        for c in range(self.nc):
            x = self.roots[c]
            nf, first = 0, {}                                    # filters walked; width -> filters before its cut
            while x.i < self.iters:
                self._expand(x)
                if x.neg:
                    y = x.kids[0]
                    self._commit(c, x, y, False, False)
                elif x.result is None:
                    break
                else:
                    r = self._rank.get(id(x), -1)                # -1: evaluated in an earlier round
                    for kk in widths:
                        if kk not in first and r >= kk:
                            first[kk] = nf
                    y = self._decision(x)
                    ok = x.result[1] == _lib.STATUS_OK
                    self.degenerate += 0 if ok else 1
                    self.degenerate_c[c] += 0 if ok else 1
                    self._commit(c, x, y, True, ok and y is x.kids[0])
                    nf += 1
                x = y
                done += 1
            for kk in widths:
                cut[kk] += first.get(kk, nf)
            x.parent = None                                      # drop the discarded tree
            self.roots[c] = x
        return done, cut

    def initialise(self):
        super().initialise()
        self.roots = []
        for c in range(self.nc):
            stream = _Stream(self.rngs[c].get_state(), self.d, self.N)
            val = _Val(self.likelihoods[c, 0], self.loglik[c, 0], self.trajs[c, :, 0, :].copy())
            self.roots.append(_Node(c, 1, None, self.thetas[c, 0].copy(), val, stream, 0, self.fnext[c]))

    def advance(self):
        """One round: schedule, evaluate (one batched filter of up to `slots` nodes), resolve.  Returns
        (iterations committed, filters of the realised path among them)."""
        f0 = sum(self.filters_run)
        if self.tuner is not None:
            import time
            t0 = time.perf_counter()
            self.slots = self.tuner.pick([self._alpha(c) for c in range(self.nc)],
                                         [self._delta(c) for c in range(self.nc)])
        nodes = self._schedule()
        if nodes:
            self._evaluate(nodes)
        widths = [k for k in self.tuner.cands if k <= len(nodes)] if self.tuner is not None else ()
        done, cut = self._resolve(widths)
        if self.tuner is not None and nodes:
            self.tuner.record(self.slots, time.perf_counter() - t0, cut)
        self.i = min(r.i for r in self.roots)
        if self.i >= self.iters:
            self._finish()
        return done, sum(self.filters_run) - f0

    def _finish(self):
        for c in range(self.nc):
            self.fnext[c] = self.roots[c].fnext

    @property
    def tuned(self):
        """slots="auto": whether the width tuner has measured every candidate (always True for a fixed width)."""
        return self.tuner is None or self.tuner.best is not None

    def step(self):
        raise NotImplementedError("PrefetchSampler advances by rounds: use advance() or run()")

    def run(self, progress=False, on_iteration=None):
        if self.roots is None:
            self.initialise()
        bar = None
        if progress:                                            # the reference's chain bar, pmcmc.py:320-406
            from tqdm import tqdm
            bar = tqdm(total=self.iters - 1, desc="Chains", position=1)
        while self.i < self.iters:
            before = self.i
            self.advance()
            if bar is not None and self.i > before:
                i = self.i - 1
                bar.update(self.i - before)
                bar.set_postfix_str(f"accepted_theta: {self.thetas[0, i]}, "
                                    f"acceptance_ratio: {100 * self.acceptances[0] / (i + 1)}%")
            if on_iteration is not None:
                for k in range(before, self.i):
                    on_iteration(k, None)
        if bar is not None:
            bar.close()
        return self.results()
