"""dreamer_amd -- MI355X-native (gfx950) Dreamer-V3 imagination engine.

Drop-in for youngers2006/Dreamer's Python API (Dreamer, WorldModel, Agent,
Buffer, ...): the imagination hot path (RSSM/GRU, categorical prior and
posterior, reward/continue/actor/critic heads, conv encoder, H-step unroll
and its actor-critic update) runs as hand-written HIP kernels in
libdreamer_hip.so behind a C ABI (include/dreamer_hip.h)."""
from .agent import Actor, Agent, Critic  # noqa: F401
from .buffer import Buffer  # noqa: F401
from .dreamer import Dreamer  # noqa: F401
from .networks import (ContinuePredictor, Decoder, DynamicsPredictor, Encoder, RewardPredictor,  # noqa: F401
                       SequenceModel)
from .world_model import WorldModel  # noqa: F401

__version__ = "0.1.0"
