"""Configuration: the reference's `Config` attribute tree and its translation to `cn_config`.

`Config` mirrors crowd_nav/configs/config.py:9-214 of the reference (same sub-objects, same attribute
names, same defaults) so that code written against the reference config keeps working. Any object
with that attribute tree — including the reference's own `Config` — can be passed to
`make_cn_config`.
"""
import numpy as np

from . import abi


class BaseConfig(object):
    def __init__(self):
        pass


class Config(object):
    """Mirror of crowd_nav/configs/config.py:9-214 (defaults identical)."""

    test = BaseConfig()
    test.social_metrics = False

    sim = BaseConfig()
    sim.render = False
    sim.train_val_sim = ["circle_crossing", "square_crossing", "parallel_traffic", "perpendicular_traffic"]
    sim.test_sim = ["circle_crossing", "square_crossing", "parallel_traffic", "perpendicular_traffic"]
    sim.square_width = 20
    test.side_preference = any("side_pref" in s_ for s_ in sim.test_sim)
    sim.circle_radius = 6 if not test.social_metrics and not test.side_preference else 4
    sim.human_num = 5 if not test.side_preference else 1
    sim.group_human = False

    env = BaseConfig()
    env.env_name = "CrowdSimDict-v0"
    env.time_limit = 50
    env.time_step = 0.25
    env.val_size = 100
    env.test_size = 500
    if test.social_metrics:
        env.test_size = 2000
    elif test.side_preference:
        env.test_size = 200
    env.randomize_attributes = True
    env.seed = 0

    reward = BaseConfig()
    reward.time_factor = False
    reward.normalize = False
    reward.potential_based = True
    reward.exponential = False
    reward.norm_zones = False
    reward.success_reward = 10 if not reward.normalize else 1
    reward.collision_penalty = -20 if not reward.normalize else -1
    reward.timeout_penalty = -20 if not reward.normalize else -1
    reward.discomfort_dist_front = 0.25
    reward.discomfort_dist_back = 0.25
    reward.discomfort_penalty_factor = 10 if not reward.normalize else 0.5
    reward.discomfort_penalty_factor *= env.time_step
    reward.potential_factor = 2 if not reward.normalize else 0.1
    reward.exp_factor = 0.5 if not reward.normalize else 0.025
    reward.exp_denom = 6
    reward.gamma = 0.99
    reward.norm_zone_side = "lhs"
    reward.norm_zone_penalty = -0.5

    humans = BaseConfig()
    humans.visible = True
    humans.policy = "orca"
    humans.radius = 0.3
    humans.v_pref = 1
    humans.sensor = "coordinates"
    humans.FOV = 2.0
    humans.random_goal_changing = True if not test.side_preference else False
    humans.goal_change_chance = 0.25
    humans.end_goal_changing = True if not test.side_preference else False
    humans.end_goal_change_chance = 1.0
    humans.random_radii = False
    humans.random_v_pref = False
    humans.random_unobservability = False
    humans.unobservable_chance = 0.3
    humans.random_policy_changing = False

    robot = BaseConfig()
    robot.visible = False
    robot.policy = "srnn"
    robot.radius = 0.3
    robot.v_pref = 1
    robot.sensor = "coordinates"
    robot.FOV = 2.0

    noise = BaseConfig()
    noise.add_noise = False
    noise.type = "uniform"
    noise.magnitude = 0.1

    lidar = BaseConfig()
    lidar.enable = False
    lidar.viz = False
    lidar.cfg = {"max_range": 5, "num_beams": 180, "robot_radius": robot.radius}

    action_space = BaseConfig()
    action_space.kinematics = "holonomic"

    orca = BaseConfig()
    orca.neighbor_dist = 10
    orca.safety_space = 0.15
    orca.time_horizon = 5
    orca.time_horizon_obst = 5

    sf = BaseConfig()
    sf.A = 2.0
    sf.B = 1
    sf.KI = 1

    social = BaseConfig()
    social.min_personal_space = 0.2
    social.max_walking_speed = 1.5

    ppo = BaseConfig()
    ppo.num_mini_batch = 2
    ppo.num_steps = 30
    ppo.recurrent_policy = True
    ppo.epoch = 5
    ppo.clip_param = 0.2
    ppo.value_loss_coef = 0.5
    ppo.entropy_coef = 0.0
    ppo.use_gae = True
    ppo.gae_lambda = 0.95

    SRNN = BaseConfig()
    SRNN.human_node_rnn_size = 128
    SRNN.human_human_edge_rnn_size = 256
    SRNN.human_node_input_size = 3
    SRNN.human_human_edge_input_size = 2
    SRNN.human_node_output_size = 256
    SRNN.human_node_embedding_size = 64
    SRNN.human_human_edge_embedding_size = 64
    SRNN.attention_size = 64

    training = BaseConfig()
    training.lr = 4e-5
    training.eps = 1e-5
    training.alpha = 0.99
    training.max_grad_norm = 0.5
    training.num_env_steps = 10e6
    training.use_linear_lr_decay = False
    training.save_interval = 200
    training.log_interval = 20
    training.use_proper_time_limits = False
    training.cuda_deterministic = False
    training.cuda = True
    training.num_processes = 12
    training.output_dir = "data/dummy"
    training.resume = False
    training.load_path = None
    training.overwrite = True
    training.num_threads = 1


class UnsupportedConfig(ValueError):
    pass


def make_cn_config(config, num_envs, env_offset=0, nenv=None, phase=None, seed=None, max_tries=1000,
                   scenarios=None, scenario_mode=None, rng=None):
    """Translate a reference-style config into `cn_config` for `num_envs` envs starting at global
    index `env_offset`; `nenv` is the reference's num_processes over all shards (make_env's envNum,
    pytorchBaselines/a2c_ppo_acktr/envs.py:66-73); `phase` defaults like make_env ('train' if nenv > 1).
    `rng` ('mt19937' default = the reference's numpy draws, or 'philox' = fast mode with the same draw
    order and distributions; also read from `config.env.rng` when set) selects the reset / goal-change
    random stream."""
    nenv = num_envs if nenv is None else nenv
    if phase is None:
        phase = "train" if nenv > 1 else "test"
    bad = []
    if getattr(config.sim, "group_human", False):
        bad.append("sim.group_human (group environment) is not part of the engine")
    if getattr(config.humans, "random_unobservability", False):
        bad.append("humans.random_unobservability")
    if getattr(config.humans, "random_policy_changing", False):
        bad.append("humans.random_policy_changing (uses the unseeded python random module)")
    if getattr(config.noise, "add_noise", False):
        bad.append("noise.add_noise")
    # lidar.enable: the LiDAR scan only feeds the 'convgru' observation, built outside the step kernel by
    # cn_lidar_obs (CrowdNavVecEnv); with the srnn policy it changes nothing the reference returns
    if not config.reward.potential_based or getattr(config.reward, "exponential", False):
        bad.append("reward.exponential")
    if config.humans.policy not in ("orca", "social_force"):
        bad.append("humans.policy=%r" % config.humans.policy)
    if config.robot.policy not in ("srnn", "convgru"):
        bad.append("robot.policy=%r (the srnn observation dict and the convgru LiDAR row are produced)"
                   % config.robot.policy)
    if config.action_space.kinematics not in ("holonomic", "unicycle"):
        bad.append("action_space.kinematics=%r" % config.action_space.kinematics)
    if bad:
        raise UnsupportedConfig("; ".join(bad))

    c = abi.CnConfig()
    c.num_envs = int(num_envs)
    c.human_num = int(config.sim.human_num)
    c.env_offset = int(env_offset)
    c.nenv = int(nenv)
    c.seed = int(config.env.seed if seed is None else seed)
    c.phase = abi.PHASES[phase]
    c.kinematics = abi.HOLONOMIC if config.action_space.kinematics == "holonomic" else abi.UNICYCLE
    c.human_policy = abi.POLICY_ORCA if config.humans.policy == "orca" else abi.POLICY_SOCIAL_FORCE
    if scenarios is None:
        scenarios = config.sim.train_val_sim if phase in ("train", "val") else config.sim.test_sim
    if isinstance(scenarios, str):
        raise TypeError("config.sim.train_val_sim or config.sim.test_sim should be a list of strings")
    if not 0 < len(scenarios) <= abi.MAX_SCENARIOS:
        raise UnsupportedConfig("1..%d scenarios supported" % abi.MAX_SCENARIOS)
    c.num_scenarios = len(scenarios)
    for k, s in enumerate(scenarios):
        c.scenarios[k] = abi.SCENARIO_ID[s]
    if scenario_mode is None:
        scenario_mode = abi.SCMODE_SEQUENTIAL if config.test.social_metrics else abi.SCMODE_ROUND_ROBIN
    c.scenario_mode = scenario_mode
    c.val_size = int(config.env.val_size)
    c.test_size = int(config.env.test_size)
    c.time_step = float(config.env.time_step)
    c.time_limit = float(config.env.time_limit)
    c.circle_radius = float(config.sim.circle_radius)
    c.square_width = float(config.sim.square_width)
    c.robot_radius = float(config.robot.radius)
    c.robot_vpref = float(config.robot.v_pref)
    c.robot_fov = float(np.pi * config.robot.FOV)
    c.human_radius = float(config.humans.radius)
    c.human_vpref = float(config.humans.v_pref)
    c.human_fov = float(np.pi * config.humans.FOV)
    c.robot_visible = int(bool(config.robot.visible))
    c.randomize_attributes = int(bool(config.env.randomize_attributes))
    c.random_goal_changing = int(bool(config.humans.random_goal_changing))
    c.end_goal_changing = int(bool(config.humans.end_goal_changing))
    c.random_radii = int(bool(config.humans.random_radii))
    c.random_v_pref = int(bool(config.humans.random_v_pref))
    c.goal_change_chance = float(getattr(config.humans, "goal_change_chance", 0.25))
    c.end_goal_change_chance = float(getattr(config.humans, "end_goal_change_chance", 1.0))
    c.success_reward = float(config.reward.success_reward)
    c.collision_penalty = float(config.reward.collision_penalty)
    c.discomfort_dist = float(config.reward.discomfort_dist_back)
    c.discomfort_penalty_factor = float(config.reward.discomfort_penalty_factor)
    c.potential_factor = float(config.reward.potential_factor)
    c.norm_zone_penalty = float(getattr(config.reward, "norm_zone_penalty", -0.5))
    c.potential_based = 1
    c.time_factor = int(bool(config.reward.time_factor))
    c.norm_zones = int(bool(getattr(config.reward, "norm_zones", False)))
    c.norm_zone_lhs = int("lhs" in getattr(config.reward, "norm_zone_side", "lhs"))
    c.min_personal_space = float(config.social.min_personal_space)
    c.max_walking_speed = float(config.social.max_walking_speed)
    c.social_metrics = int(bool(config.test.social_metrics))
    c.side_preference = int(bool(config.test.side_preference))
    c.orca_neighbor_dist = float(config.orca.neighbor_dist)
    c.orca_safety_space = float(config.orca.safety_space)
    c.orca_time_horizon = float(config.orca.time_horizon)
    c.orca_time_horizon_obst = float(config.orca.time_horizon_obst)
    c.sf_A = float(config.sf.A)
    c.sf_B = float(config.sf.B)
    c.sf_KI = float(config.sf.KI)
    c.max_tries = int(max_tries)
    rng = getattr(config.env, "rng", "mt19937") if rng is None else rng
    if rng not in abi.RNG_MODE:
        raise UnsupportedConfig("rng=%r (one of %s)" % (rng, sorted(abi.RNG_MODE)))
    c.rng_mode = abi.RNG_MODE[rng]
    return c


def clone_config(config):
    """Independent copy of a reference-style config (the reference keeps its sub-configs as CLASS
    attributes, so two `Config()` instances share state; the clone gets instance-level copies)."""
    import copy

    new = Config.__new__(Config)
    for name in dir(config):
        if name.startswith("_"):
            continue
        val = getattr(config, name)
        if type(val).__name__ == "BaseConfig":
            setattr(new, name, copy.deepcopy(val))
    return new


def make_mixed_cn_configs(scenario_configs, scenarios, num_envs, env_offset=0, nenv=None, phase=None, rng=None):
    """Per-env scenario dispatch with per-env human counts for CrowdNavEngine.mixed.

    `scenarios` is the round-robin scenario list: env r (global index env_offset + r) runs
    scenarios[(env_offset + r) % len(scenarios)] (the engine's deterministic stand-in for the reference's
    per-reset `random.choices`, crowd_sim_dict.py:110-125). `scenario_configs` maps each scenario name to
    the reference-style config its envs use (human_num, circle_radius, test.side_preference, goal
    changing, ... -- e.g. the side_pref_* scenarios at N = 1, crowd_sim.py:334-357,642-651); scenarios
    that share one config object share one group. Returns (list of cn_config, env_group int32 [num_envs])."""
    nenv = num_envs if nenv is None else nenv
    keys, groups, env_group = [], [], np.zeros(num_envs, np.int32)
    for s in scenarios:
        if id(scenario_configs[s]) not in keys:
            keys.append(id(scenario_configs[s]))
            groups.append(scenario_configs[s])
    sc_group = [keys.index(id(scenario_configs[s])) for s in scenarios]
    for r in range(num_envs):
        env_group[r] = sc_group[(env_offset + r) % len(scenarios)]
    cfgs = [make_cn_config(c, num_envs=int((env_group == g).sum()), env_offset=env_offset, nenv=nenv, phase=phase,
                           scenarios=list(scenarios), scenario_mode=abi.SCMODE_ROUND_ROBIN, rng=rng)
            for g, c in enumerate(groups)]
    return cfgs, env_group
