"""Reference module name `Dreamer` (drop-in for train_car_racer.py); see INTEGRATION.md."""
from dreamer_amd.dreamer import Dreamer  # noqa: F401
