def dict_to_obs(d):
    return d


def obs_space_info(space):
    raise NotImplementedError


def obs_to_dict(obs):
    return obs
