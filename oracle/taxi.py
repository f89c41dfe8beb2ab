"""ORACLE / TEST INFRASTRUCTURE — numpy restatement of the batched (PO-)Taxi hot path
(`gym_po/envs/extended_taxi.py`), plus an exact computation of its reset distribution.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may use this module.
"""
import math

import numpy as np

from .draws import NumpyDraws
from .gridworld import load_maps

ACTIONS_YX = np.array([[-1, 0], [1, 0], [0, -1], [0, 1], [0, 0]])  # extended_taxi.py:154 (N,S,W,E,PD)


def walled_map(rows):
    """extended_taxi.py:57-70 — pad with '|'; pseudo-wall maps navigate every other column."""
    desc = np.pad(np.asarray(rows, dtype="c").astype(str), 1, constant_values="|")
    if (desc == ":").any():
        return desc, desc[1:-1, 1:-1:2], (lambda r, c: (r + 1, 2 * c + 1))
    return desc, desc[1:-1, 1:-1], (lambda r, c: (r + 1, c + 1))


def hansen_map(desc, tgrid, cc):
    """extended_taxi.py:102-114 — wall bits N=1, S=2, W=4, E=8."""
    h = np.zeros(tgrid.shape, dtype=int)
    w = (desc == "|").astype(int)
    for r in range(h.shape[0]):
        for c in range(h.shape[1]):
            br, bc = cc(r, c)
            h[r, c] = w[br - 1, bc] + 2 * w[br + 1, bc] + 4 * w[br, bc - 1] + 8 * w[br, bc + 1]
    return h


def resolve_map(map):
    maps = load_maps()
    if map in (None, "TAXI"):
        return maps["taxi_map"]
    if map == "EXTENDED":
        return maps["extended_taxi_map"]
    return list(map)


class TaxiOracle:
    """TaxiVecEnv restated (extended_taxi.py:149-372)."""
    STATE_ALIASES = dict(s="s", elapsed="elapsed", n_dropoffs="n_dropoffs_completed")

    def __init__(self, num_envs=1, time_limit=200, num_passengers=1, map="TAXI", hansen_obs=False,
                 reward_goal=1.0, reward_bad=-0.5, reward_any=-0.05):
        self.num_envs = num_envs
        self.GOAL_MOVE, self.BAD_MOVE, self.ANY_MOVE = reward_goal, reward_bad, reward_any
        self.desc, self.tgrid, self.cc = walled_map(resolve_map(map))
        self.hansen_encodings = hansen_map(self.desc, self.tgrid, self.cc)
        self.rows, self.cols = self.tgrid.shape
        locs = np.nonzero((self.tgrid != "|") & (self.tgrid != " ") & (self.tgrid != ":"))
        self.np_locs = np.array(locs).T
        self.nlocs = self.np_locs.shape[0]
        self.np_locs = np.concatenate((self.np_locs, [[-1, -1]]))
        self.time_limit = time_limit
        self.elapsed = np.zeros(num_envs, dtype=int)
        self.ns = self.rows * self.cols * self.nlocs * (self.nlocs + 1)
        self.no = (16 if hansen_obs else self.rows * self.cols) * self.nlocs * (self.nlocs + 1)
        self.valid_states = np.array([self.encode(r, c, p, d) for r in range(self.rows) for c in range(self.cols)
                                      if self.tgrid[r, c] != "|" for p in range(self.nlocs)
                                      for d in range(self.nlocs) if d != p])
        self.state_distribution = np.zeros(self.ns)
        self.state_distribution[self.valid_states] += 1
        self.state_distribution /= self.state_distribution.sum()
        self.hansen = hansen_obs
        self.n_dropoffs = num_passengers
        self.s = np.zeros(num_envs, dtype=int)
        self.n_dropoffs_completed = np.zeros(num_envs)

    def encode(self, r, c, p, d):
        """extended_taxi.py:97-99."""
        return ((r * self.cols + c) * (self.nlocs + 1) + p) * self.nlocs + d

    def decode(self, s):
        """extended_taxi.py:84-94."""
        d = s % self.nlocs
        t = s // self.nlocs
        p = t % (self.nlocs + 1)
        t = t // (self.nlocs + 1)
        return (t // self.cols).astype(int), (t % self.cols).astype(int), p.astype(int), d.astype(int)

    def reset_seed(self, seed):
        self.gen = np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))
        return self.reset(NumpyDraws(self.gen))

    def reset(self, draws):
        self._reset_mask(np.ones(self.num_envs, bool), draws)
        return self.obs()

    def step_seeded(self, action):
        return self.step(action, NumpyDraws(self.gen))

    def step(self, actions, draws):
        """extended_taxi.py:244-287."""
        self.elapsed += 1
        r, c, p, d = self.decode(self.s)
        a = ACTIONS_YX[actions]
        rn = np.clip(r + a[:, 0], 0, self.rows - 1)
        cn = np.clip(c + a[:, 1], 0, self.cols - 1)
        cc = self.cc(rn, cn)
        ok = self.desc[cc] != "|"
        crossed = a[:, 1].astype(bool) & (self.desc[cc[0], cc[1] - a[:, 1]] == "|")
        ok &= ~crossed
        r[ok], c[ok] = rn[ok], cn[ok]
        tloc = np.column_stack((r, c))
        rew = np.full(self.num_envs, self.ANY_MOVE, dtype=np.float32)
        pd = actions == 4
        goal = pd & (p == self.nlocs) & (self.np_locs[d] == tloc).all(-1)
        self.n_dropoffs_completed[goal] += 1
        pick = pd & (p < self.nlocs) & (self.np_locs[p] == tloc).all(-1)
        p[pick] = self.nlocs
        self.s = self.encode(r, c, p, d)
        bad = pd & ~goal & ~pick
        rew[goal] = self.GOAL_MOVE
        rew[bad] = self.BAD_MOVE
        done = np.zeros(self.num_envs, bool)
        done[self.n_dropoffs_completed == self.n_dropoffs] = True
        trunc = self.elapsed > self.time_limit
        task = goal & ~(done | trunc)
        self._reset_pd(task, r[task], c[task], draws)
        self._reset_mask(done | trunc, draws)
        return self.obs(), rew, done, trunc

    def _reset_mask(self, mask, draws):
        """extended_taxi.py:344-352."""
        if mask.sum():
            self.s[mask] = draws.multinomial_argmax(self.ns, self.state_distribution, mask, "reset_state")
            self.elapsed[mask] = 0
            self.n_dropoffs_completed[mask] = 0

    def _reset_pd(self, mask, r, c, draws):
        """extended_taxi.py:354-364 — p uniform, d resampled while d == p."""
        b = int(mask.sum())
        if b:
            if isinstance(draws, NumpyDraws):
                p_idx = draws.integers(self.nlocs, b, "p")
                d_idx = draws.integers(self.nlocs, b, "d")
                while (m := mask[mask] & (p_idx == d_idx)).any():
                    d_idx[m] = draws.integers(self.nlocs, int(m.sum()), "d")
            else:
                pd = draws.a["pd"][mask]
                p_idx, d_idx = pd // self.nlocs, pd % self.nlocs
            self.s[mask] = self.encode(r, c, p_idx, d_idx)

    def obs(self):
        """extended_taxi.py:366-372."""
        if not self.hansen:
            return self.s.copy()
        r, c, p, d = self.decode(self.s)
        return (self.hansen_encodings[r, c] * (self.nlocs + 1) + p) * self.nlocs + d


def argmax_multinomial_distribution(m, n, c_max=None):
    """P(argmax = k), k = 0..m-1, for counts ~ Multinomial(n, uniform over m bins), ties -> first.

    Exact up to float64 rounding, via Poissonization: with N_j iid Poisson(n/m), the counts
    conditioned on sum = n are that multinomial, so
      P(argmax=k) = sum_c pois(c) [x^(n-c)] Q_{c-1}(x)^k Q_c(x)^(m-1-k) / P(sum=n),
    Q_b(x) = sum_{i<=b} pois(i) x^i. This is the start-state law of TaxiVecEnv._reset_mask
    (extended_taxi.py:344-352: multinomial(ns, uniform over the valid states).argmax()).
    """
    lam = n / m
    if c_max is None:
        c_max = min(n, int(lam + 40))
    pois = np.array([math.exp(-lam + i * math.log(lam) - math.lgamma(i + 1)) for i in range(n + 1)])
    p_sum_n = math.exp(-n + n * math.log(n) - math.lgamma(n + 1))
    out = np.zeros(m)
    for c in range(1, c_max + 1):
        q_lo = pois[:c].copy()       # Q_{c-1}
        q_hi = pois[:c + 1].copy()   # Q_c
        deg = n - c
        if deg < 0:
            break
        pw_lo = np.zeros((m, deg + 1))
        pw_hi = np.zeros((m, deg + 1))
        pw_lo[0, 0] = pw_hi[0, 0] = 1.0
        for k in range(1, m):
            pw_lo[k] = np.convolve(pw_lo[k - 1], q_lo)[:deg + 1]
            pw_hi[k] = np.convolve(pw_hi[k - 1], q_hi)[:deg + 1]
        # coefficient of x^deg in pw_lo[k] * pw_hi[m-1-k]
        coef = np.einsum("ki,ki->k", pw_lo, pw_hi[::-1][:, ::-1])
        out += pois[c] * coef
    return out / p_sum_n
