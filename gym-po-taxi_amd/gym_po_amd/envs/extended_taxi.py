"""(PO-)Taxi — drop-in for `gym_po.envs.extended_taxi` (pending)."""
from functools import partial

from ..maps import EXTENDED_TAXI_MAP, TAXI_MAP


class TaxiVecEnv:
    def __init__(self, *a, **k):
        raise NotImplementedError("TaxiVecEnv backend pending")


HansenTaxiVecEnv = partial(TaxiVecEnv, hansen_obs=True)
ExtendedTaxiVecEnv = partial(TaxiVecEnv, map=EXTENDED_TAXI_MAP)
ExtendedHansenTaxiVecEnv = partial(HansenTaxiVecEnv, map=EXTENDED_TAXI_MAP)
