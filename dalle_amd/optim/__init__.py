from .lamb import LAMB8bit, CPULAMB8Bit, LambWithGradientClipping  # noqa: F401
from .flat import FlatArena  # noqa: F401
from .schedule import get_linear_schedule_with_warmup  # noqa: F401
