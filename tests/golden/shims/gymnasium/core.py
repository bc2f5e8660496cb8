class Env(object):
    spec = None

    def reset(self, seed=None, options=None):
        return None
