"""Environment wrappers with the reference's class names (Adaptors.py).
Env-side CPU code, outside the imagination hot path.  gymnasium / PyFlyt are
imported lazily so importing this module never requires them (the reference
hard-imports cv2 and PyFlyt, Adaptors.py:3-4)."""
import numpy as np

try:
    import gymnasium as gym
    _Action, _Obs, _Wrap = gym.ActionWrapper, gym.ObservationWrapper, gym.Wrapper
except ImportError:  # pragma: no cover - exercised only without gymnasium
    gym = None

    class _Missing:
        def __init__(self, *a, **k):
            raise ImportError("gymnasium is required for the environment adaptors")

    _Action = _Obs = _Wrap = _Missing


class DroneAdaptor(_Action):  # Adaptors.py:6-22
    def __init__(self, env):
        super().__init__(env)
        self.action_space = gym.spaces.Box(low=-1, high=1, shape=(4,), dtype=np.float32)

    def action(self, action):
        return np.array([action[0], action[1], action[2], action[3]], dtype=np.float32)


class CarRacerAdaptor(_Action):  # Adaptors.py:24-33: gas/brake mapped from [-1,1] to [0,1]
    def __init__(self, env):
        super().__init__(env)
        self.action_space = gym.spaces.Box(low=-1, high=1, shape=(3,), dtype=np.float32)

    def action(self, action):
        return np.array([action[0], (action[1] + 1) / 2, (action[2] + 1) / 2])


class CropObservation(_Obs):  # Adaptors.py:35-46: keep the top 84 rows (drop the dashboard)
    def __init__(self, env):
        super().__init__(env)
        self.observation_space = gym.spaces.Box(low=0, high=255, shape=(84, 96, 3), dtype=np.uint8)

    def observation(self, obs):
        return obs[:84, :, :]


class ActionRepeat(_Wrap):  # Adaptors.py:48-69
    def __init__(self, env, repeat=4):
        super().__init__(env)
        self.repeat = repeat

    def step(self, action):
        total, done, trunc, obs, info = 0.0, False, False, None, {}
        for _ in range(self.repeat):
            obs, r, d, t, info = self.env.step(action)
            total += r
            done, trunc = done or d, trunc or t
            if done or trunc:
                break
        return obs, total, done, trunc, info
