class Monitor(object):
    def __init__(self, env, filename, allow_early_resets=False):
        self.env = env
