"""primesim_amd — MI355X-native uncore timing engine for PriME's memory-system hot path.

The product is the HIP engine in libprimeuncore.so (C ABI: include/primeuncore.h);
this package is its Python host mirror (`uncore.UncoreManager`), the config_prime
schema (`config`) and the ctypes ABI definitions (`_abi`).
"""
from . import _abi, config  # noqa: F401
from .uncore import (InsMem, StreamSet, StreamSpec, UncoreError, UncoreManager, config_from_dict,  # noqa: F401
                     generate_stream, load_config, msglog_from_stream, msglog_read, parse_config,
                     stream_threads, MsgLogWriter)

__all__ = ["InsMem", "StreamSet", "StreamSpec", "UncoreError", "UncoreManager", "config_from_dict", "generate_stream",
           "load_config", "msglog_from_stream", "msglog_read", "MsgLogWriter", "parse_config", "stream_threads"]
