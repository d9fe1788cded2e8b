"""avt_amd — MI355X-native audio-visual hard-way train step (drop-in for
tonymisic/audio-visual-tubes model.py / train_hardway_1frame.py).

Import through the repo-root shim: ``import avtubes`` (registers this directory as ``avt_amd``).
"""
__version__ = "0.1.0"
