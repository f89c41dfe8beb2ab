from .crooms import CRoomsEnv
from .msrooms import MultistoryFourRoomsEnv
from .rooms import RoomsEnv
