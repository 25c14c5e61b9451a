"""Reference module name `Adaptors` (drop-in for train_car_racer.py); see INTEGRATION.md."""
from dreamer_amd.adaptors import DroneAdaptor, CarRacerAdaptor, CropObservation, ActionRepeat  # noqa: F401
