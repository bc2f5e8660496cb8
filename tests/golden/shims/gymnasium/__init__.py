"""Minimal gymnasium stand-in (gymnasium is absent in this image).

Only what the reference's env modules touch at import/construct/step time:
`core.Env`, `spaces.{Text,Box,Dict,Sequence}`, `spaces.discrete.Discrete` and
`envs.registration.register`.  Golden-vector generation only; none of it
touches game arithmetic.
"""
from . import core, spaces, envs  # noqa: F401
