"""GEMM API over the gfx950 MFMA tile engine, plus the reference's GEMM benchmark.

``myGEMM`` keeps the reference contract (fpcode/gpu_func.cu:259, inc/gpu_func.h:44-47):
column-major, ``C := alpha * op(A) * op(B) + beta * C`` -- with all four
transpose combinations honoured (the reference silently ignores BT when AT is
set, gpu_func.cu:263-273).  ``gemm`` is the same operation on row-major torch
tensors.  ``benchmark_gemm`` reproduces BenchmarkGEMM (fpcode/utils/tests.cpp:
77-280): deterministic createMATS inputs, alpha=2, beta=5, a warm-up then 10
accumulating iterations of the library GEMM (hipBLAS/hipBLASLt through torch)
and of ours, max-norm relative difference <= 1e-12 in fp64.
"""
from __future__ import annotations

import time

import torch

from .._native import hip

_CODES = {torch.float32: 0, torch.float64: 1, torch.bfloat16: 2}
GEMM_TOL = 1e-12  # fpcode/utils/tests.cpp:13
NUM_ITERS = 10    # fpcode/utils/tests.cpp:12


def _code(t: torch.Tensor) -> int:
    if t.dtype not in _CODES:
        raise TypeError(f"unsupported dtype {t.dtype}")
    return _CODES[t.dtype]


def _check(*ts):
    for t in ts:
        if not t.is_cuda:
            raise ValueError("GEMM operands must be on the GPU")
        if not t.is_contiguous():
            raise ValueError("GEMM operands must be contiguous")
    if len({t.dtype for t in ts}) != 1:
        raise TypeError("GEMM operands must share one dtype")


def myGEMM(A: torch.Tensor, B: torch.Tensor, C: torch.Tensor, alpha: float, beta: float, M: int, N: int, K: int,
           AT: bool = False, BT: bool = False) -> int:
    """Reference-style column-major GEMM on flat device buffers; returns 0 (as myGEMM)."""
    _check(A, B, C)
    lda = K if AT else M
    ldb = N if BT else K
    if A.numel() < M * K or B.numel() < K * N or C.numel() < M * N:
        raise ValueError("operand buffers too small for the requested GEMM")
    hip().gemm(_code(A), bool(AT), bool(BT), M, N, K, float(alpha), A.data_ptr(), lda, B.data_ptr(), ldb,
               float(beta), C.data_ptr(), M, torch.cuda.current_stream(A.device).cuda_stream)
    return 0


def gemm(A: torch.Tensor, B: torch.Tensor, C: torch.Tensor | None = None, alpha: float = 1.0, beta: float = 0.0,
         transA: bool = False, transB: bool = False) -> torch.Tensor:
    """Row-major ``C = alpha * op(A) @ op(B) + beta * C`` on the MFMA engine."""
    M = A.shape[1] if transA else A.shape[0]
    K = A.shape[0] if transA else A.shape[1]
    N = B.shape[0] if transB else B.shape[1]
    if (B.shape[1] if transB else B.shape[0]) != K:
        raise ValueError("inner dimensions differ")
    if C is None:
        C = torch.zeros(M, N, dtype=A.dtype, device=A.device)
        beta = 0.0
    _check(A, B, C)
    # row-major C (M x N) is the column-major matrix C^T (N x M) = op(B)^T op(A)^T
    hip().gemm(_code(A), bool(transB), bool(transA), N, M, K, float(alpha), B.data_ptr(),
               K if transB else N, A.data_ptr(), M if transA else K, float(beta), C.data_ptr(), N,
               torch.cuda.current_stream(A.device).cuda_stream)
    return C


def create_mats(M: int, N: int, K: int, dtype=torch.float64, device="cuda"):
    """createMATS (tests.cpp:77-99), column-major flat buffers."""
    i = torch.arange(M, dtype=torch.float64).view(M, 1)
    k = torch.arange(K, dtype=torch.float64)
    A = (i * k.view(1, K) / M).t().contiguous().view(-1)            # A[i + j*M] = i*j/M
    kk = torch.arange(K, dtype=torch.float64).view(K, 1)
    j = torch.arange(N, dtype=torch.float64).view(1, N)
    B = ((kk * j + 1) / N).t().contiguous().view(-1)                 # B[i + j*K] = (i*j+1)/N
    C = ((i * j + 2) / N).t().contiguous().view(-1)                  # C2[i + j*M] = (i*j+2)/N
    return (A.to(dtype).to(device), B.to(dtype).to(device), C.to(dtype).to(device))


def _inf_norm_colmajor(x: torch.Tensor, M: int, N: int) -> float:
    return float(x.view(N, M).t().abs().sum(dim=1).max())


def test_gemm(M: int, N: int, K: int, dtype=torch.float64, device="cuda", iters: int = NUM_ITERS,
              verbose: bool = True) -> dict:
    """TestGEMM (tests.cpp:126-259) vs the vendor BLAS (hipBLAS/hipBLASLt via torch)."""
    A, B, C = create_mats(M, N, K, dtype, device)
    alpha, beta = 2.0, 5.0
    Am = A.view(K, M).t()
    Bm = B.view(N, K).t()

    def lib_step(Cf):
        Cm = Cf.view(N, M).t()
        r = torch.addmm(Cm, Am, Bm, beta=beta, alpha=alpha)  # library GEMM
        Cf.view(N, M).t().copy_(r)

    C_ref = C.clone()
    C_mine = C.clone()
    lib_step(C.clone())  # warm-up
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        lib_step(C_ref)
    torch.cuda.synchronize()
    t_ref = time.perf_counter() - t
    myGEMM(A, B, C.clone(), alpha, beta, M, N, K)  # warm-up
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        myGEMM(A, B, C_mine, alpha, beta, M, N, K)
    torch.cuda.synchronize()
    t_mine = time.perf_counter() - t
    rel = _inf_norm_colmajor((C_mine - C_ref).double(), M, N) / _inf_norm_colmajor(C_ref.double(), M, N)
    tol = {torch.float64: GEMM_TOL, torch.float32: 1e-5, torch.bfloat16: 3e-2}[dtype]
    flops = 2.0 * M * N * K * iters
    res = dict(M=M, N=N, K=K, dtype=str(dtype).replace("torch.", ""), rel_diff=rel, ok=rel <= tol,
               lib_s=t_ref, mine_s=t_mine, lib_tflops=flops / t_ref / 1e12, mine_tflops=flops / t_mine / 1e12)
    if verbose:
        status = "matched with reference successfully!" if res["ok"] else "output not matching with reference."
        print(f"GEMM {M}x{N}x{K} {res['dtype']}: {status} Rel diff = {rel:.3e}")
        print(f"  Time for reference (vendor BLAS) GEMM implementation: {t_ref:.6f} seconds")
        print(f"  Time for my GEMM implementation: {t_mine:.6f} seconds")
    return res


def benchmark_gemm(device="cuda", shapes=((800, 1000, 784), (800, 10, 1000)), dtypes=(torch.float64,),
                   verbose: bool = True) -> list:
    """BenchmarkGEMM (tests.cpp:261-280): the two reference shapes (plus any extra)."""
    out = []
    for dt in dtypes:
        for (M, N, K) in shapes:
            out.append(test_gemm(M, N, K, dt, device, verbose=verbose))
    return out
