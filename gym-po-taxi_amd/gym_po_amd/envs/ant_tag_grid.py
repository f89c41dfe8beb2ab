"""Grid Ant-Tag (build-defined restatement of ant_tag.py task rules). (pending)"""


class AntTagGridEnv:
    def __init__(self, *a, **k):
        raise NotImplementedError("AntTagGridEnv backend pending")
