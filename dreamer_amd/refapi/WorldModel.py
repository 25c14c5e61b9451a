"""Reference module name `WorldModel` (drop-in for train_car_racer.py); see INTEGRATION.md."""
from dreamer_amd.world_model import WorldModel  # noqa: F401
