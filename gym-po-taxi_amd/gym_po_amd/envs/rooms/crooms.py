"""C-ROOMS — drop-in for `gym_po.envs.rooms.crooms.CRoomsEnv` (crooms.py:91-338). (pending)"""


class CRoomsEnv:
    def __init__(self, *a, **k):
        raise NotImplementedError("CRoomsEnv backend pending")
