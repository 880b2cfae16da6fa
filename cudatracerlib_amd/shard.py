"""Image-tile sharding across GPUs.

Rank r of N owns the 64x64 tiles with ``tile_id % N == r`` (interleaved for
load balance; tile space of IBlockSampler.h:100-108).  A *step* renders N
progressive passes on every rank, so per-GPU work is fixed (weak scaling) and
after K steps the job holds the N*K-pass image.  Pixel i always uses sampler
index y*w+x and the same pass index, so every sample equals the 1-GPU one.
A jittered sample can round over a tile border onto another rank's pixel
(AddSample adds at floor(x + u)); the rank that owns the target pixel traces
that path itself (apron work items, a few per image) and sums each of its
pixels in the 1-GPU order, so the per-rank PixelData framebuffers are
disjoint and one reduce gives exactly the 1-GPU image.
"""


def shard_params(params, world, rank):
    """Point a ctl_pt_params (PTParams) at this rank's tiles."""
    params.num_ranks = int(world)
    params.rank = int(rank)
    return params


def step_pass_indices(step, world, base=0):
    """Sampler pass indices rendered by every rank in `step`."""
    return [base + step * world + k for k in range(world)]


def owned_tiles(width, height, tile, world, rank):
    tiles = (-(-width // tile)) * (-(-height // tile))
    return [t for t in range(tiles) if t % world == rank]


def reduce_framebuffer(fb, dist, dst=0, out=None):
    """Sum the per-rank PixelData framebuffers into a separate image on `dst`
    (RCCL over xGMI on GPUs, gloo on CPU) and return it (on `dst`; other ranks
    get their send copy back).  Every pixel is nonzero on its owner rank only,
    so the fp32 sum is exact: x + 0 = x.  `fb` itself is never written: each rank
    keeps accumulating its own pixels, so this may run after any step (a
    reduce in place would fold the other ranks' totals into dst's accumulator
    and count them again at the next reduce)."""
    if fb.is_cuda and dist.get_backend() == "gloo":
        # gloo reduces host tensors only (CPU rehearsals of the N-rank path)
        host = fb.cpu()
        dist.reduce(host, dst=dst, op=dist.ReduceOp.SUM)
        if out is None:
            return host.to(fb.device)
        out.copy_(host)
        return out
    if out is None:
        out = fb.clone()
    else:
        out.copy_(fb)
    dist.reduce(out, dst=dst, op=dist.ReduceOp.SUM)
    return out
