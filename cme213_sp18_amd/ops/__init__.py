"""Op-level Python API over the gfx950 kernels (GEMM, MLP pieces)."""
