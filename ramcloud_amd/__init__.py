"""ramcloud_amd -- MI355X-native CRC32C integrity-checksum path of RAMCloud.

Product: libramcrc.so (HIP kernels for gfx950 + C ABI, include/ramcrc.h) and the
drop-in C++ headers in include/ramcloud/.  This package holds the HIP/C++
sources (csrc/), the build script, a ctypes binding and the multi-GPU
recovery-scan driver.
"""
__all__ = ["ramcrc", "workloads", "recovery_scan", "build"]
