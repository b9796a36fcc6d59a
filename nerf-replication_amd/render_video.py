"""360-degree turntable render (reference: render_video.py:21-70).

    python render_video.py --cfg_file configs/nerf/lego.yaml [video_frames 240]
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 render_video.py \
        --cfg_file configs/nerf/lego.yaml

The reference's 240 poses (pose_spherical(angle, -30, 4) for angle in linspace(-180, 180,
241)[:-1]) are rendered with Renderer.render, rays generated on the GPU (nerf_raygen).
Under torch.distributed.run every frame's rays are split across the GPUs and gathered
(src/utils/dist_render.py).  Rank 0 writes result_dir/video_frames/frame_XXX.png and, when
imageio is importable, the reference's <exp_name>_360_video_60fps.mp4 (imageio is not in
this image; the PNG frames are always written).  Without the test dataset on disk the
camera comes from the config (test_dataset.H/W, the lego camera_angle_x).
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from src.config import cfg  # noqa: E402


def _camera():
    """(H, W, focal) of the test split (the reference builds a test Dataset for this)."""
    try:
        from src.datasets.nerf.blender import Dataset
        ds = Dataset(**cfg.test_dataset)
        return ds.H, ds.W, ds.focal
    except (FileNotFoundError, OSError):
        from src.utils.camera import focal_for
        r = float(cfg.test_dataset.get("input_ratio", 1.0))
        H, W = int(cfg.test_dataset.H * r), int(cfg.test_dataset.W * r)
        return H, W, focal_for(int(cfg.test_dataset.W)) * r


def video_poses(n, device=None):
    """The reference's turntable: pose_spherical(angle, -30, 4) for angle in linspace(-180, 180,
    n + 1)[:-1] (render_video.py:46-49)."""
    from src.utils.camera import pose_spherical
    return torch.stack([pose_spherical(float(a), -30.0, 4.0) for a in np.linspace(-180, 180, n + 1)[:-1]]).to(device)


def render_frame(renderer, pose, H, W, focal, near, far, pix=None):
    """One frame (render_video.py:53-64): the camera's rays (nerf_raygen), Renderer.render (split
    over the ranks under torchrun), rgb_map_f (else rgb_map_c) -> (float [H,W,3], uint8 [H,W,3]
    = clip(rgb, 0, 1) * 255 truncated, as the reference's numpy cast), both on the device."""
    from nerf_amd import ops
    from src.utils.dist_render import render_distributed
    if pix is None:
        pix = torch.arange(H * W, device=pose.device)
    with torch.no_grad():
        rays, _, _ = ops.raygen(pose.reshape(1, 4, 4), H, W, focal, pix=pix)
        out = render_distributed(renderer, {"rays": rays, "near": near, "far": far}, keys=("rgb_map_f", "rgb_map_c"))
    rgb = out.get("rgb_map_f", out["rgb_map_c"]).reshape(H, W, 3)
    return rgb, rgb.clamp(0, 1).mul(255).to(torch.uint8)


def render_360_video(num_frames=None, write=True):
    from nerf_amd import ops
    from src.models import make_network
    from src.models.nerf.renderer.make_renderer import make_renderer
    from src.utils.net_utils import load_network

    rank = 0
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        import torch.distributed as dist
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        if not dist.is_initialized():
            dist.init_process_group("nccl", init_method="env://", device_id=torch.device("cuda", local))
        rank = dist.get_rank()
    device = torch.device("cuda", torch.cuda.current_device())
    network = make_network(cfg)
    load_network(network, cfg.trained_model_dir, resume=True)
    network.to(device).eval()
    renderer = make_renderer(cfg, network)
    n = int(num_frames or cfg.get("video_frames", 240))
    poses = video_poses(n, device)
    H, W, focal = _camera()
    near = ops.device_scalar(float(cfg.task_arg.near), device)
    far = ops.device_scalar(float(cfg.task_arg.far), device)
    pix = torch.arange(H * W, device=device)
    out_dir = os.path.join(cfg.result_dir, "video_frames")
    if rank == 0 and write:
        os.makedirs(out_dir, exist_ok=True)
    frames, t0 = [], time.time()
    for i in range(n):
        _, img = render_frame(renderer, poses[i], H, W, focal, near, far, pix)
        if rank != 0:
            continue
        frames.append(img.cpu().numpy())
        if write:
            from PIL import Image
            Image.fromarray(frames[-1]).save(os.path.join(out_dir, f"frame_{i:03d}.png"))
    if rank == 0:
        dt = time.time() - t0
        print(f"rendered {n} frames of {H}x{W} in {dt:.2f} s ({dt / max(n, 1):.4f} s/frame)")
        if write:
            try:
                import imageio
                path = os.path.join(cfg.result_dir, f"{cfg.exp_name}_360_video_60fps.mp4")
                imageio.mimsave(path, frames, fps=30, quality=8)
                print(f"video saved to {path}")
            except ImportError:
                print(f"imageio is not installed: frames are in {out_dir}")
    return frames


if __name__ == "__main__":
    render_360_video()
