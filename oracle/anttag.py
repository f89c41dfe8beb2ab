"""ORACLE / TEST INFRASTRUCTURE — numpy restatement of the build-defined grid Ant-Tag.

The reference's Ant-Tag (gym_po/envs/ant_tag.py:88-157) is a MuJoCo robot task; only its tag
rules are restated, on a grid, by the build (spec in gym-po-taxi_amd/csrc/anttag.hip and DESIGN.md).
There is no reference output to pin this oracle against: parity unpinned with respect to the
reference; the oracle pins the device kernel to the build's own spec (replay and philox modes,
bit-exact), and tests/test_oracle_anttag.py checks the spec's laws on the CPU.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may use this module.
"""
import numpy as np

from .philox import env_step_words, lemire_value

TAG = 0x616E7431
DY = np.array([-1, 0, 1, 0, 0])  # N, E, S, W, stay
DX = np.array([0, 1, 0, -1, 0])


class AntTagOracle:
    STATE_ALIASES = dict(ant="ant", target="target", elapsed="elapsed")

    def __init__(self, num_envs, size=10, tag_radius2=2, visible_radius2=9, min_start_dist2=25, time_limit=500,
                 tag_reward=1.0, step_reward=0.0):
        self.B, self.N = num_envs, size
        self.tag_r2, self.vis_r2, self.min_r2 = tag_radius2, visible_radius2, min_start_dist2
        self.time_limit = time_limit
        self.tag_reward, self.step_reward = np.float32(tag_reward), np.float32(step_reward)
        nc = size * size
        cy, cx = np.divmod(np.arange(nc), size)
        d2 = (cy[:, None] - cy[None, :]) ** 2 + (cx[:, None] - cx[None, :]) ** 2
        self.valid_targets = [np.flatnonzero(d2[a] > min_start_dist2) for a in range(nc)]
        self.ant = np.zeros(num_envs, np.int64)
        self.target = np.zeros(num_envs, np.int64)
        self.elapsed = np.zeros(num_envs, np.int64)

    # ---- draws: philox (device counter layout) or replay arrays ----
    def philox_draws(self, step, key):
        x0, x1, x2, _ = env_step_words(self.B, step, TAG, key)
        choose = (x0 >> np.uint32(30)).astype(np.int64)
        ant = lemire_value(x1, self.N * self.N)
        cnt = np.array([len(v) for v in self.valid_targets])[ant]
        k = ((x2.astype(np.uint64) * cnt.astype(np.uint64)) >> np.uint64(32)).astype(np.int64)  # Lemire, n = cnt
        return dict(choose=choose, ant=ant, tgt=k)

    def _reset(self, mask, dr):
        ant = dr["ant"][mask]
        k = dr["tgt"][mask]
        tgt = np.array([self.valid_targets[a][min(kk, len(self.valid_targets[a]) - 1)] for a, kk in zip(ant, k)],
                       dtype=np.int64)
        self.ant[mask] = ant
        self.target[mask] = tgt
        self.elapsed[mask] = 0

    def reset(self, dr):
        self._reset(np.ones(self.B, bool), dr)
        return self.obs()

    def obs(self):
        ay, ax = np.divmod(self.ant, self.N)
        ty, tx = np.divmod(self.target, self.N)
        vis = (ay - ty) ** 2 + (ax - tx) ** 2 < self.vis_r2
        return np.stack([ay, ax, np.where(vis, ty, -1), np.where(vis, tx, -1)], -1).astype(np.int32)

    def step(self, actions, dr):
        N = self.N
        self.elapsed += 1
        a = np.asarray(actions, dtype=np.int64)
        a = np.where(a < 0, a + 5, a).clip(0, 4)
        ay, ax = np.divmod(self.ant, N)
        ty, tx = np.divmod(self.target, N)
        ny, nx = ay + DY[a], ax + DX[a]
        ok = (ny >= 0) & (ny < N) & (nx >= 0) & (nx < N)
        ay, ax = np.where(ok, ny, ay), np.where(ok, nx, ax)
        dy, dx = ay - ty, ax - tx
        c = dr["choose"] & 3
        vy = np.select([c == 0, c == 1, c == 2], [-dy, -dx, dx], 0)
        vx = np.select([c == 0, c == 1, c == 2], [-dx, dy, -dy], 0)
        avy, avx = np.abs(vy), np.abs(vx)
        sy = np.where(avy >= avx, np.sign(vy), 0)
        sx = np.where(avx >= avy, np.sign(vx), 0)
        my, mx = ty + sy, tx + sx
        ok = (my >= 0) & (my < N) & (mx >= 0) & (mx < N)
        ty, tx = np.where(ok, my, ty), np.where(ok, mx, tx)
        self.ant, self.target = ay * N + ax, ty * N + tx
        d2 = (ay - ty) ** 2 + (ax - tx) ** 2
        term = d2 <= self.tag_r2
        rew = np.where(term, self.tag_reward, self.step_reward).astype(np.float32)
        trunc = self.elapsed >= self.time_limit
        mask = term | trunc
        if mask.any():
            self._reset(mask, dr)
        return self.obs(), rew, term, trunc
