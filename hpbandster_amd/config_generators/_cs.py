"""ConfigSpace binding: the real package when installed, else the engine's compatible stand-in."""
try:  # pragma: no cover - depends on the environment
    import ConfigSpace  # noqa: F401
except ImportError:  # ConfigSpace is not part of this image
    from .. import configspace as ConfigSpace  # noqa: F401
