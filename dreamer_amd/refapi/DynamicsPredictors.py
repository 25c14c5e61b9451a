"""Reference module name `DynamicsPredictors` (drop-in for train_car_racer.py); see INTEGRATION.md."""
from dreamer_amd.networks import DynamicsPredictor, RewardPredictor, ContinuePredictor  # noqa: F401
