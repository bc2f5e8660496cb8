class Discrete(object):
    def __init__(self, n, seed=None, start=0):
        self.n = int(n)
        self.start = start
        self.shape = ()
