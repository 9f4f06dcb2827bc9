"""MI355X-native batched CrowdSimDict engine + DSRNN policy (drop-in for CrowdNav_DSRNN's env/policy hot path).

  crowdnav_dsrnn_amd.envs.make_vec_envs   VecEnv adapter registered as 'CrowdSimDict-v0'
  crowdnav_dsrnn_amd.engine.CrowdNavEngine device-resident batched env (C ABI: include/crowdnav.h)
  crowdnav_dsrnn_amd.policy.Policy        DSRNN actor-critic with the reference's state_dict keys
"""
