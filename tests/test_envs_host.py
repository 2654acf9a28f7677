"""CPU tests of the Atari preprocessing (origin_repo/wrapper.py): the stage
adapters under the reference's wrapper names on a scripted emulator, the wrapped synthetic
Atari env's observation contract (Q10: H/W transposed, raw 0..255), and the vectorised
``AtariPreprocess`` pipeline reproducing the composed wrapper stack step for step."""
import numpy as np
import pytest

from apex_amd.envs import atari
from apex_amd.envs.core import Env
from apex_amd.envs.spaces import Box, Discrete


class Scripted(Env):
    """Emulator stub: frame t is filled with t; rewards and lives follow a script."""

    def __init__(self, rewards=None, lives=None, done_at=None, shape=(210, 160, 3)):
        super().__init__()
        self.observation_space = Box(0, 255, shape=shape, dtype=np.uint8)
        self.action_space = Discrete(4)
        self.rewards, self.lives_script, self.done_at = rewards or {}, lives or {}, done_at
        self.ale = self
        self.n_resets, self.actions = 0, []
        self.reset()

    def get_action_meanings(self):
        return ["NOOP", "FIRE", "UP", "DOWN"]

    def lives(self):
        return self._lives

    def _obs(self):
        return np.full(self.observation_space.shape, self.t % 256, np.uint8)

    def reset(self):
        self.t, self._lives = 0, 3
        self.n_resets += 1
        return self._obs()

    def step(self, action):
        self.actions.append(int(action))
        self.t += 1
        self._lives = self.lives_script.get(self.t, self._lives)
        done = self.done_at is not None and self.t >= self.done_at
        return self._obs(), float(self.rewards.get(self.t, 0.0)), done, {}


def test_max_and_skip_repeats_action_and_maxes_last_two():
    env = atari.MaxAndSkipEnv(Scripted(rewards={2: 1.0, 4: 2.0, 6: 5.0}), skip=4)
    env.reset()
    obs, r, done, _ = env.step(3)
    assert env.env.actions == [3] * 4 and r == 3.0 and not done
    assert obs.max() == 4 and obs.min() == 4  # max(frame 3, frame 4)
    obs, r, _, _ = env.step(1)
    assert r == 5.0 and obs.min() == 8
    # a done inside the skip window ends the repeat early
    env = atari.MaxAndSkipEnv(Scripted(done_at=2), skip=4)
    env.reset()
    _, _, done, _ = env.step(0)
    assert done and len(env.env.actions) == 2


def test_clip_reward_is_sign():
    env = atari.ClipRewardEnv(Scripted(rewards={1: 20.0, 2: -3.0}))
    env.reset()
    assert [env.step(0)[1] for _ in range(3)] == [1.0, -1.0, 0.0]


def test_warp_frame_area_resample():
    m = atari._area_matrix(84, 210)
    assert m.shape == (84, 210) and np.allclose(m.sum(1), 1.0) and (m >= 0).all()
    # exact 2x2 box filter when the scale is integral
    env = atari.WarpFrame(Scripted(shape=(168, 168, 3)))
    rng = np.random.default_rng(0)
    frame = rng.integers(0, 256, (168, 168, 3)).astype(np.uint8)
    out = env.observation(frame)
    gray = frame.astype(np.float64) @ np.array([0.299, 0.587, 0.114])
    ref = gray.reshape(84, 2, 84, 2).mean((1, 3))
    assert out.shape == (84, 84, 1) and out.dtype == np.uint8
    assert np.abs(out[..., 0].astype(np.float64) - ref).max() <= 0.5 + 1e-9
    assert (atari.WarpFrame(Scripted()).observation(np.full((210, 160, 3), 77, np.uint8)) == 77).all()


def test_episodic_life_ends_on_life_loss_without_reset():
    env = atari.EpisodicLifeEnv(Scripted(lives={3: 2}))
    env.reset()
    dones = [env.step(0)[2] for _ in range(3)]
    assert dones == [False, False, True] and not env.ledger.game_over
    n = env.env.n_resets
    env.reset()  # life lost, game not over: a NOOP step, not an emulator reset
    assert env.env.n_resets == n and env.env.actions[-1] == 0 and env.lives == 2


def test_noop_and_fire_reset():
    env = atari.NoopResetEnv(Scripted(), noop_max=30)
    env.fixed_noops = 5
    env.reset()
    assert env.env.actions == [0] * 5
    env = atari.FireResetEnv(Scripted())
    env.reset()
    assert env.env.actions == [1, 2]


def test_frame_stacks_and_image_to_pytorch():
    env = atari.FrameStack(atari.WarpFrame(Scripted()), 4)
    ob = env.reset()
    for _ in range(2):
        ob, _, _, _ = env.step(0)
    a = np.asarray(ob)
    assert a.shape == (84, 84, 4) and list(a[0, 0]) == [0, 0, 1, 2]
    env = atari.TorchFrameStack(atari.ImageToPyTorch(atari.WarpFrame(Scripted())), 4)
    ob = env.reset()
    ob, _, _, _ = env.step(0)
    a = np.asarray(ob)
    assert a.shape == (4, 84, 84) and list(a[:, 0, 0]) == [0, 0, 0, 1]
    assert env.observation_space.shape == (4, 84, 84)


@pytest.mark.parametrize("game", ["Seaquest", "Pong"])
def test_wrapped_synthetic_atari_contract(game):
    from apex_amd.config import preset

    cfg = preset("origin").env
    env = atari.wrap_atari_dqn(atari.make_atari(f"{game}NoFrameskip-v4"), cfg)
    env.seed(3)
    ob = np.asarray(env.reset())
    assert ob.shape == (4, 84, 84) and ob.dtype == np.uint8
    total = 0.0
    for t in range(200):
        ob, r, done, _ = env.step(env.action_space.sample())
        assert r in (-1.0, 0.0, 1.0)  # clipped
        total += abs(r)
        if done:
            ob = env.reset()
    assert np.asarray(ob).shape == (4, 84, 84)


@pytest.mark.parametrize("game,episode_life,scale", [("Seaquest", 1, 0), ("Pong", 1, 0), ("Breakout", 0, 1)])
def test_vector_pipeline_matches_wrapper_stack(game, episode_life, scale):
    """AtariPreprocess over N emulators == N independent make_atari + wrap_atari_dqn stacks:
    same observations, clipped rewards, life-loss dones and restarts."""
    from types import SimpleNamespace

    from apex_amd.envs.preprocess import AtariPreprocess, PreprocessSpec
    from apex_amd.envs.core import make

    args = SimpleNamespace(episode_life=episode_life, clip_rewards=1, frame_stack=1, scale=scale)
    env_id = f"{game}NoFrameskip-v4"
    N = 3
    stacks = [atari.wrap_atari_dqn(atari.make_atari(env_id), args) for _ in range(N)]
    for i, e in enumerate(stacks):
        e.seed(11 + i)
    pipe = AtariPreprocess([make(env_id) for _ in range(N)], PreprocessSpec.from_args(args))
    pipe.seed(11)
    obs_v = pipe.reset()
    obs_w = np.stack([np.asarray(e.reset()) for e in stacks])
    assert obs_v.shape == (N,) + pipe.obs_shape and np.array_equal(obs_v, obs_w)
    rng = np.random.default_rng(0)
    n_done = 0
    for t in range(300):
        acts = rng.integers(0, stacks[0].action_space.n, N)
        obs_v, r_v, d_v, _ = pipe.step(acts)
        for i, e in enumerate(stacks):
            o, r, d, _ = e.step(int(acts[i]))
            assert np.array_equal(obs_v[i], np.asarray(o)), (t, i)
            assert r_v[i] == r and d_v[i] == d
            if d:
                n_done += 1
                assert np.array_equal(pipe.reset_one(i), np.asarray(e.reset()))
    assert obs_v.dtype == (np.float32 if scale else np.uint8)
    if episode_life and game != "Pong":  # Pong has no lives (21-point games)
        assert n_done > 0  # life losses and the restarts after them were exercised


def test_repeat_pool_terminal_frames_match_the_reference_buffer():
    """origin_repo/wrapper.py:99-124 keeps a persistent two-slot buffer written only at
    repeat steps skip-2 and skip-1: a window that ends early returns the max of frames from
    EARLIER windows.  RepeatPool(reference=True) pins that; reference=False is the
    this-window max."""
    import numpy as np

    from apex_amd.envs.preprocess import RepeatPool

    def stepper(dones):
        it = iter(dones)
        k = [0]

        def step(_a):
            k[0] += 1
            return np.full((2, 2), k[0], dtype=np.uint8), 1.0, next(it), {}
        return step

    ref, win = RepeatPool(4), RepeatPool(4, reference=False)
    # window 1: frames 1..4, slots <- (3, 4); window 2 ends at its first step (frame 5)
    dones = [False] * 4 + [True]
    s_ref, s_win = stepper(dones), stepper(dones)
    assert int(ref.run(s_ref, 0)[0].max()) == 4 and int(win.run(s_win, 0)[0].max()) == 4
    f_ref, r_ref, d_ref, _ = ref.run(s_ref, 0)
    f_win, _, _, _ = win.run(s_win, 0)
    assert d_ref and r_ref == 1.0
    assert int(f_ref.max()) == 4   # stale slots of window 1 (the reference's behaviour)
    assert int(f_win.max()) == 5   # this window's only frame
    # a window ending at step skip-2 (third frame) overwrites slot 0 only: max(slot0 new, slot1 old)
    p = RepeatPool(4)
    s = stepper([False] * 4 + [False, False, True])
    p.run(s, 0)                       # slots (3, 4)
    f, _, d, _ = p.run(s, 0)          # frames 5, 6, 7(done at i=2): slot0 <- 7, slot1 stays 4
    assert d and int(f.max()) == 7 and int(f.min()) == 7
    p2 = RepeatPool(4)
    s2 = stepper([False] * 4 + [False, True])
    p2.run(s2, 0)
    f2, _, _, _ = p2.run(s2, 0)       # frames 5, 6(done at i=1): slots untouched -> max(3, 4)
    assert int(f2.max()) == 4
