from . import registration  # noqa: F401

registry = registration.registry
