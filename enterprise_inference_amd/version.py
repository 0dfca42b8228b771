__version__ = "0.1.0"
# Reference release this stack is capability-compatible with (core/version.txt:2-3).
REFERENCE_VERSION = "1.3.0"
