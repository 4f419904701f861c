"""PTv3 device ops (placeholder; filled in with the PTv3 kernels)."""
