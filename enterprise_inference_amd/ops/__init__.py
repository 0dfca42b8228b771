"""Fused ops: HIP kernels on the GPU (csrc/kernels), PyTorch references on the CPU."""
