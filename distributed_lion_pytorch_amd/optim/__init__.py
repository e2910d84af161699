from .lion import Lion  # noqa: F401
