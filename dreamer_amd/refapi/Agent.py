"""Reference module name `Agent` (drop-in for train_car_racer.py); see INTEGRATION.md."""
from dreamer_amd.agent import Agent, Actor, Critic  # noqa: F401
