"""lbwn — MI355X-native WaveNet hot path (hrbigelow/lb-wavenet drop-in).

Host side of the C-ABI library liblbwn.so: arch/par surface, the WaveNetTrain /
WaveNetGen classes, the µ-law ops, the slice dealer and checkpoints.
"""
__version__ = '0.1.0'
