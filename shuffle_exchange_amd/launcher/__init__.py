"""Launcher (parity: reference launcher/): ``python -m shuffle_exchange_amd.launcher.runner`` or ``bin/sxe``."""
