"""hpbandster_amd: MI355X-native engine for HpBandSter's KDE acquisition + SH promotion path."""
__version__ = "0.1.0"
