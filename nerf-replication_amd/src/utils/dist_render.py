"""Multi-GPU inference: one image's rays dealt to the ranks in interleaved blocks (block b
to rank b mod W), rendered independently, then gathered (640,000 rays / 8 =
80,000 per GPU; rgb/depth/acc gathered at the end, no other collective).  Interleaving keeps
the ranks' work equal when it is not uniform over the image: the grid march
(render_accelerated, volume_renderer.py:268-357) queries the MLP only where rays cross
occupied cells, which cluster in the central rows, so contiguous row blocks would leave the
middle ranks with most of the frame.  The grid bake: one voxel slab per rank (16 x 128 x 128
at 8 ranks), then an all-gather of the bool grid (2 MB).

Used by run.py --type evaluate|network under torch.distributed.run; the renderer is any
object with render / render_accelerated (the reference's Renderer interface)."""
import torch
import torch.distributed as dist


def _world():
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def shard_bounds(n: int, rank: int, world: int):
    """[start, stop) of rank's contiguous share of n rays (sizes differ by at most one)."""
    return n * rank // world, n * (rank + 1) // world


RAY_BLOCK = 256  # rays per dealt block (640,000-ray frame: 2,500 blocks, 312-313 per rank at 8)


def interleaved_index(n: int, rank: int, world: int, block: int = RAY_BLOCK, device=None):
    """Ray ids of rank's share: blocks b = rank, rank + W, ... of ``block`` consecutive rays."""
    nb = (n + block - 1) // block
    blocks = torch.arange(rank, nb, world, device=device)
    idx = (blocks[:, None] * block + torch.arange(block, device=device)[None]).reshape(-1)
    return idx[idx < n]


def ray_block(n: int, world: int, block: int = RAY_BLOCK) -> int:
    """Rays per dealt block: ``block``, shrunk for small images so that every rank gets at
    least one block whenever n >= world (a 40x40 view on 8 ranks: 200-ray blocks)."""
    return max(1, min(block, -(-n // world)))


def _meta(out, n_mine, keys):
    """{key: ("ray", tail shape, dtype) | ("scalar", type name, None) | ("other", None, None)}
    of a rank's render output, in the output's key order (the order every rank then walks the
    keys in).  Per-ray tensors outside ``keys`` are dropped."""
    m = {}
    for k, v in out.items():
        if torch.is_tensor(v) and v.dim() >= 1 and v.shape[0] == n_mine:
            if keys is None or k in keys:
                m[k] = ("ray", tuple(v.shape[1:]), v.dtype)
        elif isinstance(v, (int, float)):
            m[k] = ("scalar", type(v).__name__, None)
        else:
            m[k] = ("other", None, None)
    return m


def render_distributed(renderer, batch, accelerated: bool = False, keys=None, block: int = RAY_BLOCK):
    """Render batch['rays'] split across ranks; every rank returns the full outputs.

    Rank r renders the rays of interleaved_index(n, r, W, ray_block(n, W, block)); per-ray
    outputs ([N] or [N, c] tensors) are padded to the largest share, all_gathered and
    scattered back to ray order; scalars (render_time, n_queried) are max- / sum-reduced.
    Every rank issues the same collectives in the same order: a rank whose share is empty
    (n < W) does not render, and the ranks first agree on the output keys (an object
    all-gather, only in that case) so it joins every gather with a [0, ...] part."""
    world = _world()
    fn = renderer.render_accelerated if accelerated else renderer.render
    if world == 1:
        return fn(batch)
    rank = dist.get_rank()
    rays = batch["rays"]
    flat = rays.reshape(-1, 6)
    n = flat.shape[0]
    blk = ray_block(n, world, block)
    idx = [interleaved_index(n, r, world, blk, flat.device) for r in range(world)]
    mine = idx[rank]
    out = {}
    if mine.numel() > 0:
        sub = dict(batch)
        own = flat.index_select(0, mine)
        sub["rays"] = own[None] if rays.dim() == 3 else own
        out = fn(sub)
    meta = _meta(out, mine.numel(), keys)
    if min(int(i.numel()) for i in idx) == 0:
        metas = [None] * world
        dist.all_gather_object(metas, meta)
        meta = next((m for m in metas if m), {})
    share = max(int(i.numel()) for i in idx)
    res = {}
    for k, (kind, info, dtype) in meta.items():
        if k not in out:  # this rank rendered nothing
            if kind == "ray":
                out[k] = torch.zeros((0,) + info, dtype=dtype, device=flat.device)
            elif kind == "scalar":
                out[k] = 0 if info == "int" else 0.0
        v = out.get(k)
        if kind == "ray":
            pad = torch.zeros((share,) + tuple(v.shape[1:]), dtype=v.dtype, device=v.device)
            pad[: mine.numel()] = v
            parts = [torch.empty_like(pad) for _ in range(world)]
            dist.all_gather(parts, pad)
            full = torch.empty((n,) + tuple(v.shape[1:]), dtype=v.dtype, device=v.device)
            for r in range(world):
                full[idx[r].to(v.device)] = parts[r][: idx[r].numel()]
            res[k] = full
        elif isinstance(v, (int, float)):
            dev = flat.device if flat.device.type != "cpu" or dist.get_backend() == "gloo" else "cuda"
            t = torch.tensor([float(v)], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.SUM if k in ("n_queried", "n_evaluated") else dist.ReduceOp.MAX)
            res[k] = type(v)(t.item())
        else:
            res[k] = v
    return res


def bake_distributed(bake_slab, res: int):
    """Occupancy bake split into x-slabs: rank r bakes voxels shard_bounds(res, r, W) with
    ``bake_slab((x0, x1)) -> bool [x1-x0, res, res]``; the slabs are all-gathered (uint8,
    padded to the largest share) so every rank returns the full bool [res, res, res] grid."""
    world = _world()
    if world == 1:
        return bake_slab((0, res))
    rank = dist.get_rank()
    a, b = shard_bounds(res, rank, world)
    part = bake_slab((a, b)).to(torch.uint8)
    share = (res + world - 1) // world
    pad = torch.zeros((share, res, res), dtype=torch.uint8, device=part.device)
    pad[: b - a] = part
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad)
    out = torch.cat([parts[r][: shard_bounds(res, r, world)[1] - shard_bounds(res, r, world)[0]]
                     for r in range(world)], 0)
    return out.bool()
