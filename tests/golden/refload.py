"""Load the read-only reference (`/root/reference/gym_po`) for golden-fixture generation.

Test infrastructure for the survey/build container ONLY:
  * prepends `refstubs/` (our own minimal gymnasium/cv2/pyglet/dotsi stand-ins) to sys.path;
  * imports `gym_po` through an importlib source hook that repairs, in memory, the 12 mangled
    parameter annotations (`nameNDArray` -> `name: np.ndarray`). Function bodies
    are untouched; nothing is written to /root/reference and no bytecode is written anywhere.

Nothing under `gym-po-taxi_amd/` imports this module; the GPU box never has /root/reference.
"""
import importlib.abc
import importlib.machinery
import importlib.util
import os
import re
import sys

REF_ROOT = os.environ.get("GYM_PO_REFERENCE", "/root/reference")
_STUBS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "refstubs")
_REPAIR = re.compile(r"\b([a-z_]+)NDArray([,)])")


class _RepairLoader(importlib.machinery.SourceFileLoader):
    def get_data(self, path):
        data = super().get_data(path)
        if path.endswith(".py"):
            src = data.decode("utf-8")
            src = _REPAIR.sub(r"\1: np.ndarray\2", src)
            return src.encode("utf-8")
        return data

    # never write .pyc next to (or for) the reference
    def set_data(self, *a, **k):
        return None

    def path_stats(self, path):
        raise OSError("no bytecode cache for the reference")


class _RepairFinder(importlib.abc.MetaPathFinder):
    def find_spec(self, fullname, path, target=None):
        if not (fullname == "gym_po" or fullname.startswith("gym_po.")):
            return None
        parts = fullname.split(".")
        base = os.path.join(REF_ROOT, *parts)
        if os.path.isdir(base):
            fn = os.path.join(base, "__init__.py")
            loader = _RepairLoader(fullname, fn)
            return importlib.util.spec_from_file_location(
                fullname, fn, loader=loader, submodule_search_locations=[base])
        fn = base + ".py"
        if os.path.exists(fn):
            loader = _RepairLoader(fullname, fn)
            return importlib.util.spec_from_file_location(fullname, fn, loader=loader)
        return None


def load():
    """Return the repaired `gym_po.envs` module namespace."""
    if not os.path.isdir(REF_ROOT):
        raise RuntimeError(f"reference not present at {REF_ROOT}")
    sys.dont_write_bytecode = True
    if _STUBS not in sys.path:
        sys.path.insert(0, _STUBS)
    if not any(isinstance(f, _RepairFinder) for f in sys.meta_path):
        sys.meta_path.insert(0, _RepairFinder())
    import gym_po.envs as envs  # noqa: E402
    import gym_po.envs.rooms.msrooms as msrooms
    import gym_po.envs.rooms.rooms as rooms
    import gym_po.envs.rooms.crooms as crooms
    import gym_po.envs.rooms.layouts as layouts
    import gym_po.envs.rooms.observations as observations
    import gym_po.envs.rooms.action_utils as action_utils
    import gym_po.envs.extended_taxi as extended_taxi
    return dict(envs=envs, msrooms=msrooms, rooms=rooms, crooms=crooms, layouts=layouts,
                observations=observations, action_utils=action_utils, extended_taxi=extended_taxi)
