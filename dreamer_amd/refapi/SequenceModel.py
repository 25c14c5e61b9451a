"""Reference module name `SequenceModel` (drop-in for train_car_racer.py); see INTEGRATION.md."""
from dreamer_amd.networks import SequenceModel  # noqa: F401
