"""Kernel bindings (``hip``) and the pure-PyTorch oracle (``reference``)."""
