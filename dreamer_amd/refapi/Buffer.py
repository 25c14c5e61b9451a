"""Reference module name `Buffer` (drop-in for train_car_racer.py); see INTEGRATION.md."""
from dreamer_amd.buffer import Buffer  # noqa: F401
