__version__ = "0.1.0"
__version_major__, __version_minor__, __version_patch__ = 0, 1, 0
# reference base: DeepSpeed 0.16.8 (+HCache fork)
reference_version = "0.16.8"
