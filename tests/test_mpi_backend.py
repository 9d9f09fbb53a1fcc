"""1-bit compressed all-reduce over the MPI transport (reference runtime/comm/mpi.py:170-290),
driven by an in-process communicator (tests/fake_mpi.py; mpi4py is not in this image, so the
real MPI library stays parity-unpinned).  Results and error-feedback state must equal the
algorithm computed directly from the same compression functions, for both transports
(device-direct "CUDA-aware" and pinned host staging), over two steps."""

import pytest
import torch

from fake_mpi import run_threads

W = 4


def _reference(ms, werrs, serrs):
    """Direct evaluation of the two-phase algorithm for all ranks (mutates the errors)."""
    from deeperspeed_amd.ops import native
    n = werrs[0].numel()
    flats = []
    for m in ms:
        f = m.reshape(-1).float()
        flats.append(torch.cat([f, torch.zeros(n - f.numel(), device=f.device)]) if f.numel() != n else f)
    packed, scales = zip(*[native.onebit_worker_compress(f.contiguous(), e) for f, e in zip(flats, werrs)])
    scales = torch.cat([s.reshape(1) for s in scales])
    chunk = packed[0].numel() // W
    sp, ss = [], []
    for s in range(W):
        recv = torch.cat([p[s * chunk:(s + 1) * chunk] for p in packed])
        a, b = native.onebit_server_compress(recv, scales, serrs[s])
        sp.append(a)
        ss.append(b.reshape(1))
    out = torch.empty(n, dtype=torch.float32, device=flats[0].device)
    native.onebit_unpack(torch.cat(sp), torch.cat(ss), out)
    return [out[:ms[0].numel()].view_as(ms[0]).to(ms[0].dtype) for _ in ms]


def _check(device, cuda_aware):
    from deeperspeed_amd.runtime.comm.mpi import MpiBackend
    n, numel = 1024, 1000
    g = torch.Generator().manual_seed(0)
    steps = [[torch.randn(numel, generator=g).to(device) for _ in range(W)] for _ in range(2)]
    werr = [torch.zeros(n, device=device) for _ in range(W)]
    serr = [torch.zeros(n // W, device=device) for _ in range(W)]
    ref_w, ref_s = [e.clone() for e in werr], [e.clone() for e in serr]

    def body(rank, comm):
        be = MpiBackend(cuda_aware=cuda_aware, comm=comm)
        outs = []
        for ms in steps:
            buf = ms[rank].clone()
            outs.append(be.compressed_allreduce(buf, werr[rank], serr[rank]).clone())
        if buf.is_cuda:
            torch.cuda.synchronize()
        return outs

    outs, comms = run_threads(W, body)
    for step, ms in enumerate(steps):
        exp = _reference([m.clone() for m in ms], ref_w, ref_s)
        for r in range(W):
            assert torch.equal(outs[r][step], exp[r]), (step, r)
    for r in range(W):
        assert torch.equal(werr[r], ref_w[r]) and torch.equal(serr[r], ref_s[r])
    # both phases post their two collectives together: alltoall+allgather, allgather+allgather
    assert [k for k, _ in comms[0].calls[:4]] == ["alltoall", "allgather", "allgather", "allgather"]
    return comms


@pytest.mark.parametrize("cuda_aware", [False, True])
def test_mpi_backend_matches_algorithm_cpu(cuda_aware):
    _check("cpu", cuda_aware)


@pytest.mark.gpu
@pytest.mark.parametrize("cuda_aware", [False, True])
def test_mpi_backend_device_paths(cuda_aware):
    comms = _check("cuda", cuda_aware)
    kinds = {t for _, t in comms[0].calls}
    # device-direct hands HIP tensors to MPI; the staged path only host (numpy) buffers
    assert kinds == ({"Tensor"} if cuda_aware else {"ndarray"})
