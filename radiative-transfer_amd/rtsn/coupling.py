"""Material-temperature coupling across group shards (include/rtsn.h,
rt_material_*; beyond the reference, whose T is constant, solver.cpp:157).

One process per GPU, each holding a block of energy groups.  Per full step
every rank sweeps its groups with the per-cell emission (B_g(T) plus the owed
emission it pays) and writes its share of the exchange term
q(x) = sum_g sigma_g (phi_g - W B_g) and of b(x) = sum_g sigma_g dB_g/dT; ONE
all-reduce (sum) of those 2N doubles over the ranks -- RCCL over xGMI on the GPU
box -- gives every rank the same [q, b], and with it the same T update
dT = dt q / (rho_cv + dt W b).  The
all-reduce is issued on the solver's own HIP stream, so sweep, collective and
update stay stream-ordered with no host synchronisation.
"""
from __future__ import annotations


def coupled_steps(solver, nsteps: int, q, world_size: int = 1, group=None, host_sync: bool = False):
    """nsteps coupled full steps of this rank's group shard.

    solver: rtsn.Solver after material_enable (or anything with its
    material_sweep(q) / material_update(q) methods); q: float64 tensor of 2N
    elements on the solver's device (the exchange buffer [q, b]); world_size > 1
    sums it over the ranks of `group` with torch.distributed.  host_sync: instead
    of ordering the all-reduce on the solver's stream, wait for the sweep on
    the host, all-reduce on the current stream and wait for it (two host
    synchronisations per step).
    """
    import torch
    import torch.distributed as dist

    stream = None
    if q.is_cuda and not host_sync:
        stream = torch.cuda.ExternalStream(solver.stream, device=q.device)
    for _ in range(int(nsteps)):
        solver.material_sweep(q)
        if world_size > 1:
            if stream is not None:
                with torch.cuda.stream(stream):
                    dist.all_reduce(q, group=group)
            else:
                if q.is_cuda:
                    solver.synchronize()
                dist.all_reduce(q, group=group)
                if q.is_cuda:
                    torch.cuda.synchronize(q.device)
        solver.material_update(q)
