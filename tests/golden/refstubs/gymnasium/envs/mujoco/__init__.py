class MujocoEnv:
    def __init__(self, *a, **k):
        pass
