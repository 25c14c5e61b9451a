"""Reference module name `VariationalAutoEncoder` (drop-in for train_car_racer.py); see INTEGRATION.md."""
from dreamer_amd.networks import Encoder, Decoder  # noqa: F401
