"""Drop-in ``network_module`` (reference: src/models/nerf/network.py:9-192).

``Network()`` reads the global cfg and owns a coarse (``model``) and a fine
(``model_fine``) NeRF MLP with the reference's parameter names, shapes, creation order
and nn.Linear init -- so ``torch.manual_seed(s); Network()`` gives the reference's
weights and ``latest.pth["net"]`` loads strictly.  ``forward(inputs [R,S,3], viewdirs
[R,3], model)`` runs the fused gfx950 kernel (positional encoding + all 11 layers,
``nerf_mlp_fwd``) and is differentiable w.r.t. the parameters through
``nerf_mlp_bwd``.  There is no PyTorch fallback: CPU tensors raise.
"""
import torch
import torch.nn as nn

from nerf_amd import ops
from src.config import cfg
from src.models.encoding import get_encoder


class NeRF(nn.Module):
    """One 8x256 NeRF MLP (network.py:9-47): parameters only; the math is the kernel."""

    def __init__(self, D=8, W=256, input_ch=63, input_ch_views=27, skips=(4,), use_viewdirs=True):
        super().__init__()
        if (D, W, input_ch, input_ch_views, tuple(skips), bool(use_viewdirs)) != (8, 256, 63, 27, (4,), True):
            raise NotImplementedError(
                "the gfx950 kernels implement the lego NeRF (D=8, W=256, skips=[4], PE 10/4 with view dirs); "
                f"got D={D} W={W} in={input_ch}/{input_ch_views} skips={list(skips)} use_viewdirs={use_viewdirs}")
        self.D, self.W = D, W
        self.input_ch, self.input_ch_views = input_ch, input_ch_views
        self.skips = list(skips)
        self.use_viewdirs = use_viewdirs
        # creation order = the reference's (seeded init parity)
        self.pts_linears = nn.ModuleList(
            [nn.Linear(input_ch, W)] + [nn.Linear(W + input_ch if i in self.skips else W, W) for i in range(D - 1)])
        self.views_linears = nn.ModuleList([nn.Linear(input_ch_views + W, W // 2)])
        self.feature_linear = nn.Linear(W, W)
        self.alpha_linear = nn.Linear(W, 1)
        self.rgb_linear = nn.Linear(W // 2, 3)
        self._packer = None

    def packer(self) -> ops.PackedMLP:
        params = ops.param_list(self)
        if self._packer is None or any(a is not b for a, b in zip(self._packer.params, params)):
            self._packer = ops.PackedMLP(params)
        return self._packer

    def forward(self, pts, viewdirs, samples_per_dir=1, dir_index=None, dtype="fp32", density_only=False):
        """raw [M,4] for points [M,3] (PE fused); view dir of point m = viewdirs[m // spd]."""
        return ops.mlp(self.packer(), pts, viewdirs, samples_per_dir, dir_index, dtype, density_only)


class Network(nn.Module):
    def __init__(self):
        super().__init__()
        ta = cfg.task_arg
        self.N_samples = ta.N_samples
        self.N_importance = ta.N_importance
        self.chunk = ta.chunk_size
        self.batch_size = ta.get("N_rays", 1024)
        self.white_bkgd = ta.white_bkgd
        self.use_viewdirs = ta.use_viewdirs
        self.mlp_dtype = ta.get("mlp_dtype", "fp32")
        self.device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
        self.embed_fn, self.input_ch = get_encoder(cfg.network.xyz_encoder)
        self.embeddirs_fn, self.input_ch_views = get_encoder(cfg.network.dir_encoder)
        n = cfg.network.nerf
        kw = dict(D=n.D, W=n.W, input_ch=self.input_ch, input_ch_views=self.input_ch_views, skips=n.skips,
                  use_viewdirs=self.use_viewdirs)
        self.model = NeRF(**kw)
        self.model_fine = NeRF(**kw)

    def mlp_dtype_for(self, model, fn):
        """The MLP arithmetic of one forward.  The bf16x3 tiers (bf16x3, bf16x3f) evaluate the
        COARSE net at fp32 when no autograd graph is recorded (render / evaluate / video):
        render()'s importance samples are a deterministic function of the coarse weights at
        perturb 0 (volume_renderer.py:82-134, u = linspace), and on the trained lego-class net a
        split-bf16 coarse MLP (~1e-5 relative per dot product) moves a sample across a CDF bin
        on a few rays of an 800x800 frame -- fine depth off by up to 3.7e-2 -- where an exact MLP
        moves them by < 1.4e-4 (tools/fullframe_conditioning.py, profiles/r5/).  With the fp32
        coarse pass every value of the frame holds the north_star's 2e-3 (tests/test_gpu_fullframe.py).
        The training forward (autograd) keeps bf16x3: at perturb 1 the importance samples are
        random draws from the CDF, which a 1e-5 relative perturbation leaves distributed the same.
        task_arg.coarse_inference_dtype (default fp32) overrides the choice: "bf16x6" (operands split exactly
        into three bf16, six products: fp32-class, faster than the fp32 MFMA) holds 2e-3 on the 4,096 sampled rays
        but leaves one frame pixel 2 uint8 levels off; "selective" (round 6) is fp32 here, while Renderer.render
        evaluates its coarse pass in the tier's arithmetic and re-evaluates at fp32 only the rays whose importance
        samples a bounded CDF perturbation could move (nerf_composite_pdf_fragile) -- measured in round 6 to need
        fp32 on 34-100 % of the frame's rays before it holds the frame's bounds (the samples move WITHIN their
        bins by dcdf / den of a bin), so neither is the default."""
        dt = self.mlp_dtype
        if model != "fine" and dt in ("bf16x3", "bf16x3f"):
            recording = torch.is_grad_enabled() and any(p.requires_grad for p in fn.parameters())
            if not recording:
                mode = cfg.task_arg.get("coarse_inference_dtype", "fp32") or dt
                # "selective" (round 6, opt-in): Renderer.render's coarse pass runs the tier's own arithmetic and
                # re-evaluates only the fragile rays at fp32 (passing dtype explicitly); any other caller of an
                # inference coarse forward gets fp32, as with "fp32"
                dt = "fp32" if mode == "selective" else mode
        return dt

    def forward(self, inputs, viewdirs, model="", dtype=None):
        """inputs [R,S,3], viewdirs [R,3] -> raw [R,S,4] (network.py:171-192); dtype overrides the MLP arithmetic."""
        fn = self.model_fine if model == "fine" else self.model
        R, S = inputs.shape[0], inputs.shape[1]
        raw = fn(inputs.reshape(-1, 3), viewdirs, S, None, dtype or self.mlp_dtype_for(model, fn))
        return raw.reshape(R, S, 4)

    def density(self, pts, model=""):
        """sigma pre-activation raw[...,3] only (the grid bake's query, occupancy_grid.py:59-60)."""
        fn = self.model_fine if model == "fine" else self.model
        return fn(pts.reshape(-1, 3), None, 1, None, self.mlp_dtype, density_only=True)[:, 3]
