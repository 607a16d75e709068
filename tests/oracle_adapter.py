"""TEST INFRASTRUCTURE: the CPU oracle behind the SimManager surface, with
zero-copy CPU torch views -- the checker the rollout harness's config-1 run
through the product's own CPU execution mode (madrona_bots.SimManager(...,
exec_mode="cpu")) is compared with.  Not a product path."""
import numpy as np
import torch

import pyoracle as po


class _T:
    def __init__(self, arr):
        self._arr = arr

    def to_torch(self):
        return torch.from_numpy(self._arr)


class OracleSimManager:
    def __init__(self, gpu_id, num_worlds, rand_seed, init_num_agents_per_world, **kw):
        self._s = po.OracleSim(num_worlds, rand_seed, init_num_agents_per_world, **kw)

    def step(self):
        self._s.step()

    def shift_observations(self):
        self._s.shift_observations()

    def _col(self, c, prev):
        return _T(self._s.column(c, prev))

    def depth_tensor(self, is_prev=False):        # exports the semantic buffer (B.1)
        return _T(self._s.column(po.COL_SEMANTIC, is_prev).view(np.uint8))

    def semantic_tensor(self, is_prev=False):
        return self._col(po.COL_SEMANTIC, is_prev)

    def reward_tensor(self, is_prev=False):
        return self._col(po.COL_REWARD, is_prev)

    def species_count_tensor(self):
        return _T(self._s.species_count())

    def position_tensor(self, is_prev=False):
        return self._col(po.COL_POS, is_prev)

    def health_tensor(self, is_prev=False):        # int32 bits as float32 (B.2)
        return _T(self._s.column(po.COL_HEALTH, is_prev).view(np.float32))

    def surrounding_tensor(self, is_prev=False):
        return self._col(po.COL_SURROUND, is_prev)

    def action_tensor(self, is_prev=False):
        return self._col(po.COL_ACTION, is_prev)

    def stats_tensor(self, is_prev=False):
        return self._col(po.COL_STATS, is_prev)

    def hidden_state_tensor(self, is_prev=False):
        return self._col(po.COL_HIDDEN, is_prev)
