"""Env classes mirroring `gym_po.envs` (gym_po/envs/__init__.py:1-4)."""
from .rooms import CRoomsEnv, MultistoryFourRoomsEnv, RoomsEnv
from .extended_taxi import (EXTENDED_TAXI_MAP, TAXI_MAP, ExtendedHansenTaxiVecEnv, ExtendedTaxiVecEnv,
                            HansenTaxiVecEnv, TaxiVecEnv)
from .ant_tag_grid import AntTagGridEnv

__all__ = ["RoomsEnv", "CRoomsEnv", "MultistoryFourRoomsEnv", "TaxiVecEnv", "HansenTaxiVecEnv",
           "ExtendedTaxiVecEnv", "ExtendedHansenTaxiVecEnv", "TAXI_MAP", "EXTENDED_TAXI_MAP", "AntTagGridEnv"]
