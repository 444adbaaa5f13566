"""MI355X-native PLDepth training hot path (HIP kernels behind the reference's Python API)."""
