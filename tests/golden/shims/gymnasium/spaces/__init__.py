class Space(object):
    def __init__(self, *args, **kwargs):
        self.args = args
        self.kwargs = kwargs
        self.shape = kwargs.get("shape")


class Text(Space):
    pass


class Box(Space):
    pass


class Dict(Space):
    pass


class Sequence(Space):
    pass


from .discrete import Discrete  # noqa: E402,F401
