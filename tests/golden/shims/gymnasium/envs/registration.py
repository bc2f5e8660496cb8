registry = {}


def register(id, **kwargs):
    registry[id] = kwargs
