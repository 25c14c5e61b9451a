"""Replay buffer with the reference's API (Buffer.py).

The host numpy ring keeps the reference's exact storage and sampling
semantics (np.random.randint starts, one redraw for windows straddling the
write head).  A device mirror of the ring (u8 frames, f32 actions, symlog
rewards, continues) lives in HBM; new transitions are uploaded lazily before
sampling, and windows are gathered on the device -- the fused train_Agent path
never materialises the float32 window at all: the encoder's first conv reads
the u8 frames straight from the ring (dr_frames)."""
import numpy as np
import torch

from . import _lib as L
from . import hip
from .utils import symlog_np


class Buffer:
    def __init__(self, buffer_size, sequence_length, action_size, observation_dims, device="cpu"):
        # observation_dims = [D]: f32 vector observations (BASELINE configs[4]); else u8 frames
        self.vector = len(tuple(observation_dims)) == 1
        self.observation_buffer = np.zeros((buffer_size, observation_dims[0]), dtype=np.float32) if self.vector \
            else np.zeros((buffer_size, 3, *observation_dims), dtype=np.uint8)
        self.action_buffer = np.zeros((buffer_size, action_size), dtype=np.float32)
        self.reward_buffer = np.zeros((buffer_size, 1), dtype=np.float32)
        self.continue_buffer = np.zeros((buffer_size, 1), dtype=np.float32)
        self.capacity = buffer_size
        self.sequence_length = sequence_length
        self.device = torch.device(device)
        self.next_idx = 0
        self.size = 0
        self._dev = None
        self._dirty = []  # slot indices not yet mirrored on the device

    # ---- host side (Buffer.py:19-30) -----------------------------------------
    def add_to_buffer(self, observation, action, reward, continue_):
        i = self.next_idx
        self.observation_buffer[i] = np.array(observation, dtype=self.observation_buffer.dtype)
        self.action_buffer[i] = np.array(action, dtype=np.float32)
        self.continue_buffer[i] = np.array(continue_, dtype=np.float32)
        self.reward_buffer[i] = symlog_np(np.array(reward, dtype=np.float32))
        self._dirty.append(i)
        self.next_idx = (i + 1) % self.capacity
        if self.size < self.capacity:
            self.size += 1

    def load_arrays(self, frames, actions, rewards_symlog, continues):
        """Bulk fill (benchmarks / fixtures): rewards already symlog'ed."""
        n = len(frames)
        assert n <= self.capacity
        self.observation_buffer[:n] = frames
        self.action_buffer[:n] = actions.reshape(n, -1)
        self.reward_buffer[:n] = rewards_symlog.reshape(n, 1)
        self.continue_buffer[:n] = continues.reshape(n, 1)
        self.size = max(self.size, n)
        self.next_idx = n % self.capacity
        self._dirty = list(range(n))

    def sample_start_indices(self, batch_size):
        """Window starts with the reference's RNG consumption (Buffer.py:33-48)."""
        if self.size < self.sequence_length:
            raise ValueError("Not enough data in buffer to sample a full sequence")
        valid = self.size - self.sequence_length + 1
        starts = np.random.randint(0, valid, size=batch_size)
        if self.size == self.capacity:
            out = []
            for s in starts:
                out.append(np.random.randint(0, valid) if s < self.next_idx < s + self.sequence_length else s)
            starts = np.array(out)
        return starts

    # ---- device mirror -------------------------------------------------------
    def _mirror(self):
        if not self.device.type == "cuda":
            raise RuntimeError("dreamer_amd: the replay device mirror needs a GPU device")
        if self._dev is None:
            self._dev = dict(
                frames=torch.zeros(self.observation_buffer.shape, dtype=torch.float32 if self.vector else torch.uint8,
                                   device=self.device),
                actions=torch.zeros(self.action_buffer.shape, device=self.device),
                rewards=torch.zeros(self.reward_buffer.shape, device=self.device),
                continues=torch.zeros(self.continue_buffer.shape, device=self.device))
            self._dirty = list(range(self.size))
        if self._dirty:
            idx = np.unique(np.asarray(self._dirty, dtype=np.int64))
            runs = np.split(idx, np.where(np.diff(idx) != 1)[0] + 1)
            for r in runs:
                a, b = int(r[0]), int(r[-1]) + 1
                for k, host in (("frames", self.observation_buffer), ("actions", self.action_buffer),
                                ("rewards", self.reward_buffer), ("continues", self.continue_buffer)):
                    self._dev[k][a:b].copy_(torch.from_numpy(host[a:b]), non_blocking=False)
            self._dirty = []
        return self._dev

    def device_key(self):
        m = self._mirror()
        return (m["frames"].data_ptr(), self.capacity)

    def frames_struct(self, starts_dev):
        """dr_frames reading the warm-start frames straight from the u8 ring
        (vector observations: the f32 ring, dr_dims.obs_dim)."""
        m = self._mirror()
        return L.dr_frames(L.ptr(m["frames"]), self.capacity, L.ptr(starts_dev), None, 0, 0, 0 if self.vector else 1)

    def gather_actions(self, starts_dev, out):
        """out[b][s][:] = action at slot (starts[b]+s) % capacity."""
        m = self._mirror()
        B, S, A = out.shape
        L.call("dr_replay_gather", self.capacity, B, S, 0, A, None, L.ptr(m["actions"]), L.ptr(m["rewards"]),
               L.ptr(m["continues"]), L.ptr(starts_dev), None, L.ptr(out), None, None, hip.stream())

    def sample_sequences(self, batch_size):
        """Buffer.sample_sequences (Buffer.py:32-63): float32 tensors on the
        buffer's device, obs holding 0..255."""
        starts = self.sample_start_indices(batch_size)
        S = self.sequence_length
        if self.device.type != "cuda":
            idx = (starts[:, None] + np.arange(S)[None, :]) % self.capacity
            f = lambda a: torch.tensor(a[idx], dtype=torch.float32, device=self.device)
            return (f(self.observation_buffer), f(self.action_buffer), f(self.reward_buffer),
                    f(self.continue_buffer), S)
        m = self._mirror()
        dev = self.device
        st = torch.as_tensor(starts, dtype=torch.int64).to(dev)
        if self.vector:  # f32 rows: a plain device gather
            idx = (st[:, None] + torch.arange(S, device=dev)[None, :]) % self.capacity
            return m["frames"][idx], m["actions"][idx], m["rewards"][idx], m["continues"][idx], S
        fe = int(np.prod(self.observation_buffer.shape[1:]))
        A = self.action_buffer.shape[1]
        obs = torch.empty(batch_size, S, *self.observation_buffer.shape[1:], device=dev)
        act = torch.empty(batch_size, S, A, device=dev)
        rew = torch.empty(batch_size, S, 1, device=dev)
        cont = torch.empty(batch_size, S, 1, device=dev)
        L.call("dr_replay_gather", self.capacity, batch_size, S, fe, A, L.ptr(m["frames"]), L.ptr(m["actions"]),
               L.ptr(m["rewards"]), L.ptr(m["continues"]), L.ptr(st), L.ptr(obs), L.ptr(act), L.ptr(rew),
               L.ptr(cont), hip.stream())
        return obs, act, rew, cont, S
