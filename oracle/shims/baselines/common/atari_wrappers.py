def make_atari(env_id):
    raise NotImplementedError


def wrap_deepmind(env, **kw):
    raise NotImplementedError
