from typing import Any
ObsType = Any
ActType = Any
RenderFrame = Any
