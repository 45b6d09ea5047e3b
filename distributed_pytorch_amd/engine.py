"""VGGEngine — the hand-scheduled MI355X trainer for the reference's VGG family.

The reference trains ``model.VGG11()`` through PyTorch autograd (main.py:31-37).  Here the whole
step is a static schedule of native kernels over persistent buffers:

  forward   per conv layer: conv_fprop (MFMA implicit GEMM, NHWC/KRSC) → bn_fwd_stats
            (batch stats + running-stat update) → bn_apply (+ReLU, +2x2 max-pool)
  head      fc_ce_train: Linear + softmax-CE loss, dlogits, dW, db, dx in two launches
  backward  per conv layer (reverse): bn_bwd (max-pool/ReLU routing recomputed from z, BN
            backward, dgamma/dbeta/dbias) → wgrad (split-K implicit GEMM) → ``grad_ready``
            callback (the gradient-sync strategy launches that bucket's collective on the comm
            stream while the remaining backward runs) → dgrad (implicit GEMM reading the weights
            with flipped taps; its split-K slabs are summed inside the next bn_bwd)
  split-K   forward/dgrad partial slabs are never reduced by a separate pass: bn_fwd_stats /
            bn_bwd sum them while computing their statistics
  update    sgd_flat over the flat parameter/grad/momentum arenas (one launch)

Parameters/grads/momentum are three :class:`~distributed_pytorch_amd.utils.arena.Arena` s with
identical layout (reference ``named_parameters()`` order; conv weights stored KRSC, the first
layer's input channels zero-padded 3→4).  ``state_dict()``/``load_state_dict()`` speak the
reference's 58-key OIHW layout (model.py; SURVEY §2.3 "Model facts").

On a CPU device the same schedule runs on :mod:`distributed_pytorch_amd.ops.cpu_ref` (plain
torch), which is what the multi-process gloo tests drive.
"""
from __future__ import annotations

import json
import os
from collections import OrderedDict
from typing import Callable, Dict, List, Optional

import torch

from . import _ext
from .models.vgg import VGGSpec
from .ops import cpu_ref
from .utils.arena import Arena
from .utils.streams import DevEvent, StreamJoin


def _pow2_round(x: float) -> int:
    p = 1
    while p * 2 <= x * 1.4142:
        p *= 2
    return p


def conv_cfg(kind: str, M: int, N: int, K: int):
    """(tile, splits) heuristic for the implicit-GEMM conv kernels, fitted to per-layer sweeps on
    MI355X (tools/conv_bench.py; profiles/conv_bench_r1.txt).  kind: 'fprop' | 'wgrad'.
    fprop/dgrad GEMM: [M x K]·[K x N];  wgrad GEMM: [N(=Kout) x M(=NPQ)]·[M x K(=RSC)]."""
    cdiv = lambda a, b: (a + b - 1) // b
    if kind == "wgrad":
        tiles = cdiv(N, 64) * cdiv(K, 64)
        s = max(1, min(128, _pow2_round(2048 / tiles)))
        while s > 1 and M // s < 128:
            s //= 2
        return 1, s
    if N <= 64:
        tiles = cdiv(M, 64) * cdiv(N, 64)
        s = 1
        while tiles * s < 512 and K // (s * 2) >= 256:
            s *= 2
        return 1, s
    tiles = cdiv(M, 128) * cdiv(N, 128)
    if tiles >= 512:
        return 0, 1
    s = max(1, _pow2_round(512 / tiles))
    while s > 1 and K // s < 256:
        s //= 2
    return 0, s


IMPLS = ("fp32", "x3", "bf16", "h2")
_TUNING = None


def tuning_table() -> Dict[str, list]:
    """Measured (tile, splits, posmajor) per conv call on MI355X (tools/tune_convs.py writes it)."""
    global _TUNING
    if _TUNING is None:
        _TUNING = {}
        p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuning", "mi355x.json")
        if os.path.exists(p) and os.environ.get("DPA_NO_TUNING", "0") != "1":
            with open(p) as f:
                _TUNING = json.load(f)
        extra = os.environ.get("DPA_TUNING_EXTRA")  # A/B of candidate entries (tools/tune_convs.py output)
        if extra:
            with open(extra) as f:
                _TUNING.update(json.load(f))
    return _TUNING


def conv_key(impl: str, kind: str, n: int, hw: int, cin: int, cout: int) -> str:
    return f"{impl}|{kind}|{n}|{hw}|{cin}|{cout}"


# Halo-staged 3x3/s1/p1 tiles of conv_x3.hip (ids after the 16 implicit-GEMM tiles): the block's
# input pixels are staged once per channel chunk and the 9 taps read shifted views of them.
HALO_TILES = (16, 17, 18, 19, 20, 21, 22, 23)  # fprop / dgrad: 256 or 128 pixels x 128 (16-19, 22) or 64
                                               # (20, 21, 23) output channels, 16-, 32- or 64-channel
                                               # chunks (22, 23: not x3's 3 planes; h2 rows <= 16 pixels)
# tile -> (rows BM, channel chunk BC) of conv_x3.hip's halo_bm / halo_bc (image slots: halo_slots)
HALO_GEOM = {16: (256, 16), 17: (256, 32), 18: (128, 16), 19: (128, 32), 20: (256, 32), 21: (128, 32),
             22: (256, 64), 23: (256, 64)}
HALO_WGRAD_TILES = (16, 17)          # wgrad: 64- or 32-pixel chunks, 128 x 32 x 9 taps per block
POS_TILES = (24, 25, 26, 27, 28, 29)  # fprop / dgrad of small images: position-major rows, padding taps
                                      # skipped (conv_x3.hip conv_pos_kernel)


def halo_ok(kind: str, tile: int, w: int, cred: int, cout: int = 8, np_: int = 2) -> bool:
    """Whether halo tile `tile` runs conv call `kind` of a 3x3/s1/p1 conv whose rows are w pixels
    wide.  cred: channels reduced (fprop C_in, dgrad C_out; wgrad C_in), cout: output channels
    (wgrad C_out), np_: operand planes (1 bf16, 2 h2, 3 x3).  Mirrors run_halo / run_halo_wgrad in
    conv_x3.hip (-6 otherwise)."""
    if kind == "wgrad":
        p = {16: 64, 17: 32}.get(tile)
        return p is not None and cred % 8 == 0 and cout % 8 == 0 and p + 2 * w + 2 <= 2 * p + 3
    if tile not in HALO_TILES:
        return False
    bm, bc = HALO_GEOM[tile]
    slots = bm + 35 if bc >= 64 and np_ >= 2 else bm + bm // 2 + 1
    if bc >= 64 and np_ == 3:
        return False
    return cred % bc == 0 and cout % 8 == 0 and bm + 2 * w + 2 <= slots - 1


def pos_ok(kind: str, tile: int, h: int, w: int, cred: int, cout: int) -> bool:
    """Whether position-major tile `tile` runs conv call `kind` (fprop / dgrad of a 3x3/s1/p1 conv)
    on h x w images; mirrors run_pos in conv_x3.hip (-6 otherwise)."""
    if kind == "wgrad" or tile not in POS_TILES or h < 2 or w < 2:
        return False
    bm = 256
    ni = 64 if tile in (26, 27, 28) else 32
    bc = 16 if tile == 29 else 32
    nspx = 4 if tile in (26, 27, 28) else 12
    ppt = bm // ni
    if (h * w) % ppt or cred % bc or cout % 8:
        return False
    worst = max((min(h, (p0 + ppt - 1) // w + 2) - max(0, p0 // w - 1)) * w for p0 in range(0, h * w, ppt))
    return worst <= nspx


class VGGEngine:
    """Static-schedule trainer.  ``impl`` selects the conv kernels of every layer whose input has a
    multiple of 8 channels (the 3-channel first layer always runs the fp32-MFMA kernel):

    * ``"fp32"`` — fp32 MFMA implicit GEMM (v_mfma_f32_32x32x2_f32), exact fp32 products;
    * ``"x3"``   — fp32-grade results on bf16 MFMA: operands kept as three bf16 planes, six plane
                   products per multiply (conv_x3.hip); error at fp32 rounding level;
    * ``"h2"``   — fp32-grade results on fp16 MFMA: operands kept as fp16 pairs of a power-of-two
                   scaled value (22 significant bits), three plane products per multiply -- half the
                   matrix work and two thirds of the operand bytes of ``"x3"`` at the same error
                   (kernels/common.h: fixed weight / activation scales with an overflow check, data
                   gradients scaled by a bound the BatchNorm backward computes every step);
    * ``"bf16"`` — one bf16 plane (mixed precision: bf16 operands, fp32 accumulation/BN/SGD).
    """

    def __init__(self, name: str = "VGG11", device="cuda", max_batch: int = 256, num_classes: int = 10,
                 lr: float = 0.1, momentum: float = 0.9, weight_decay: float = 1e-4, bn_momentum: float = 0.1,
                 bn_eps: float = 1e-5, in_hw: int = 32, backend=None, impl: str = "fp32"):
        self.device = torch.device(device)
        self.K = backend if backend is not None else (_ext.require() if self.device.type == "cuda" else cpu_ref)
        if impl not in IMPLS:
            raise ValueError(f"impl must be one of {IMPLS}")
        if self.K is cpu_ref:
            impl = "fp32"  # the CPU oracle backend implements the fp32 kernel API only
        self.impl = impl
        self.np = {"fp32": 0, "x3": 3, "bf16": 1, "h2": 2}[impl]
        pdt = torch.float16 if self.np == 2 else torch.bfloat16  # operand-plane storage
        # fp16 pairs: fixed weight / activation scales (the kernels' H2_SW / H2_SA) and per-layer
        # data-gradient bound words (bn_bwd writes them, the convs that read dz divide the scale out)
        self.h2_sw, self.h2_sa = 256.0, 16.0
        # plane kernels take the 3-channel input padded to 8 (one 16-B chunk per pixel)
        self.spec = VGGSpec.from_name(name, num_classes, in_hw, in_pad=8 if self.np else 4)
        self.max_batch = max_batch
        self._cfg_cache: Dict[tuple, tuple] = {}
        self.lr, self.momentum, self.weight_decay = lr, momentum, weight_decay
        self.bn_momentum, self.bn_eps = bn_momentum, bn_eps
        self.num_classes = num_classes
        self.steps_taken = 0
        dev = self.device
        L = self.spec.convs
        entries = []
        for l in L:
            entries += [(f"{l.conv_key}.weight", (l.cout, 3, 3, l.cin_pad)), (f"{l.conv_key}.bias", (l.cout,)),
                        (f"{l.bn_key}.weight", (l.cout,)), (f"{l.bn_key}.bias", (l.cout,))]
        entries += [("fc1.weight", (num_classes, self.spec.fc_in)), ("fc1.bias", (num_classes,))]
        self.params = Arena(entries, dev)
        self.grads = self.params.like()
        self.mom = self.params.like()
        self.buffers = Arena([(f"{l.bn_key}.{b}", (l.cout,)) for l in L for b in ("running_mean", "running_var")],
                             dev)
        self.nbt = torch.zeros(len(L), dtype=torch.int64, device=dev)
        for l in L:
            self.buffers[f"{l.bn_key}.running_var"].fill_(1.0)

        # ---- workspaces (sized for max_batch) ----
        N = max_batch
        f32 = dict(device=dev, dtype=torch.float32)
        self.x0 = torch.zeros(N, in_hw, in_hw, 4, **f32)
        # bf16 planes of the (padded) network input when layer 0 runs the plane kernels
        self.x0p = (torch.zeros(self.np, N, in_hw, in_hw, L[0].cin_pad, dtype=pdt, device=dev)
                    if self.np and L[0].cin_pad % 8 == 0 else None)
        self.target = torch.zeros(N, dtype=torch.int64, device=dev)
        bf = dict(device=dev, dtype=pdt)
        # planes(i): layer i runs the bf16-plane kernels (needs cin % 8 == 0)
        self.planes = [self.np > 0 and l.cin_pad % 8 == 0 for l in L]
        self.z, self.a, self.g, self.dz = [], [], [], []
        self.a3: List[Optional[torch.Tensor]] = []   # planes of a[i] when layer i+1 consumes planes
        self.dz3: List[Optional[torch.Tensor]] = []
        # bf16 operand planes of the WHOLE parameter arena (same element index as params.flat): the
        # fused SGD kernel rewrites them with every update; conv layer i reads its slice as w3[i]
        # (forward and, read transposed in place, data gradient)
        self.wplanes = torch.zeros(self.np, self.params.flat.numel(), **bf) if any(self.planes) else None
        self.w3: List[Optional[torch.Tensor]] = []
        self.dzb = torch.zeros(len(L), dtype=torch.int32, device=dev) if self.np == 2 else None
        self.stats = []  # per layer dict(mean, invstd, scale, shift)
        self.eval_ss = []
        part_need = 1
        for i, l in enumerate(L):
            hw, ho = l.hw, (l.hw // 2 if l.pool else l.hw)
            nxt_planes = i + 1 < len(L) and self.planes[i + 1]
            self.z.append(torch.empty(N, hw, hw, l.cout, **f32))
            self.a.append(None if nxt_planes else torch.empty(N, ho, ho, l.cout, **f32))
            self.a3.append(torch.empty(self.np, N, ho, ho, l.cout, **bf) if nxt_planes else None)
            self.g.append(torch.empty(N, ho, ho, l.cout, **f32))
            self.dz.append(None if self.planes[i] else torch.empty(N, hw, hw, l.cout, **f32))
            self.dz3.append(torch.empty(self.np, N, hw, hw, l.cout, **bf) if self.planes[i] else None)
            if self.planes[i]:
                off, cnt = self.params.offsets[f"{l.conv_key}.weight"], self.params.numels[f"{l.conv_key}.weight"]
                self.w3.append(self.wplanes[:, off:off + cnt].view(self.np, l.cout, 3, 3, l.cin_pad))
            else:
                self.w3.append(None)
            self.stats.append({k: torch.zeros(l.cout, **f32) for k in ("mean", "invstd", "scale", "shift")})
            self.eval_ss.append({k: torch.zeros(l.cout, **f32) for k in ("scale", "shift")})
            M, Mo = N * hw * hw, N * ho * ho
            part_need = max(part_need, self.K.bn_part_floats(M, l.cout, False),
                            self.K.bn_part_floats(Mo, l.cout, True))
        # Weight gradients run on a second HIP stream (DPA_WGRAD_STREAM=0: one stream): wgrad(i) needs
        # only dz(i) and the stored forward activation, so it runs beside dgrad(i) and the BN
        # backward of layer i-1, whose reduce/finalize kernels leave most CUs idle.  It has its own
        # split-K workspace.
        self.wstream = (self._make_wgrad_stream(dev) if dev.type == "cuda" and os.environ.get("DPA_WGRAD_STREAM", "1") == "1"
                        else None)
        self._wev = [DevEvent() for _ in L] if self.wstream is not None else None
        self._join = StreamJoin() if self.wstream is not None else None
        # kernel-start signals instead of per-layer events on the critical-path stream (signal.hip):
        # the data-gradient conv of layer i stores the step's epoch into ksig[i] when it starts, the
        # wgrad stream polls it.  Plane (x3 / bf16) convs only; never under graph capture (a graph may
        # order the polling kernel before its producer).  DPA_KSIGNAL=0: events everywhere.
        self.ksignal = (self.wstream is not None and os.environ.get("DPA_KSIGNAL", "1") == "1"
                        and hasattr(self.K, "wait_signal"))
        self.ksig = torch.zeros(len(L), dtype=torch.int32, device=dev) if self.ksignal else None
        self.bsig = torch.zeros(len(L), dtype=torch.int32, device=dev) if self.ksignal else None  # BN bwd starts
        self.ksig_tmo = torch.zeros(1, dtype=torch.int32, device=dev) if self.ksignal else None
        # the end-of-backward join (main waits for the wgrad stream) as a signal too: a one-wave
        # kernel on the wgrad stream stores the epoch, the main stream polls it -- an event wait on
        # the main stream idles it ~13 us even when the wgrad stream has long finished
        # (profiles/r5_h2_step_timeline.txt: the gap in front of sgd_flat).  DPA_SIGNAL_JOIN=0: event.
        self.jsig = (torch.zeros(1, dtype=torch.int32, device=dev)
                     if self.ksignal and os.environ.get("DPA_SIGNAL_JOIN", "1") == "1" else None)
        self._sig_epoch = 0
        # A wait may legitimately last as long as the main stream is held behind the previous step's
        # collectives (a slow peer: up to the communicator's DPA_COMM_TIMEOUT, after which the RCCL
        # watchdog aborts), so the bound is never shorter than that plus a minute.
        # DPA_KSIGNAL_TIMEOUT_US, when set, is taken as given (tests use short bounds).
        comm_us = int(float(os.environ.get("DPA_COMM_TIMEOUT", "600")) * 1e6)
        env_tmo = os.environ.get("DPA_KSIGNAL_TIMEOUT_US")
        self.ksig_timeout_us = int(env_tmo) if env_tmo else comm_us + 60_000_000
        # The one-launch BN's slice rendezvous waits only for blocks of its own grid (never for the
        # communicator), so it has its own short bound: a residency shortfall surfaces in seconds,
        # not after the communicator's timeout.
        self.bn_fused_timeout_us = int(os.environ.get("DPA_BN_FUSED_TIMEOUT_US", "2000000"))
        # params_free hands the sync a later kernel's signal instead of recording an event
        self.free_signal = True
        self.head_side = self.ksignal
        self.slab = torch.empty(1, **f32)
        self.wslab = torch.empty(1, **f32) if self.wstream is not None else None
        for i in range(len(L)):  # size the split-K workspaces for the full-batch plan
            for kind in ("fprop", "dgrad", "wgrad"):
                if kind == "dgrad" and i == 0:
                    continue
                self._ensure_slab(self._slab_need(i, kind, N), wgrad=kind == "wgrad" and self._wgrad_on_side(i))
        # Layer 0 (3-channel input, 32x32, 2x2 pool) has no data gradient: its BN-backward apply and
        # weight gradient run as one fused fp32 kernel (bn.hip bn_bwd_wgrad0_kernel) that never stores
        # dz.  DPA_FUSED_WGRAD0=0 runs them separately (A/B).
        l0 = L[0]
        self.fused_wgrad0 = (dev.type == "cuda" and hasattr(self.K, "bn_bwd_wgrad0")
                             and os.environ.get("DPA_FUSED_WGRAD0", "1") == "1"
                             and l0.hw == 32 and l0.cout == 64 and l0.pool and l0.cin <= 3)
        self.wpart = (torch.empty(self.K.wgrad0_part_floats(N), **f32) if self.fused_wgrad0 else None)
        # Layer 0 forward: direct fp32 conv of the 3-channel input with the BN statistics in its epilogue
        # (first_layer.hip); DPA_FUSED_CONV0=0 runs the implicit-GEMM conv + statistics pass (A/B)
        self.fused_conv0 = (dev.type == "cuda" and hasattr(self.K, "conv0_fwd")
                            and os.environ.get("DPA_FUSED_CONV0", "1") == "1"
                            and l0.hw == 32 and l0.cout == 64 and l0.cin <= 3)
        self.part0 = torch.empty(self.K.conv0_part_floats(N), **f32) if self.fused_conv0 else None
        # Head: the last layer's BN + ReLU + 2x2 max-pool folded into the classifier kernel's row load
        # (fc_ce.hip BnIn: one launch less on the critical path); DPA_FUSED_HEAD=0 runs bn_apply
        lL = L[-1]
        self.fused_head = (dev.type == "cuda" and os.environ.get("DPA_FUSED_HEAD", "1") == "1" and lL.pool
                           and lL.hw == 2 and self.spec.fc_in == lL.cout and self.a[-1] is not None)
        # One-launch BatchNorm (bn_fused.hip) for the small layers: statistics, finalize and apply
        # (forward) / reduce, finalize and apply (backward) in one kernel whose blocks meet per
        # channel slice.  Used where z has at most DPA_BN_FUSED_MAX elements (0: never) and the tile
        # geometry fits (<= DPA_BN_FUSED_RMAX row blocks per slice).  Counters self-reset; the
        # workspace is zeroed once here.
        # Defaults from same-box A/B (docs/PERF_NOTES.md, round 3): forward for z <= 2.2M elements
        # (layers 4-7 at batch 256), backward only for the 2x2 layers (<= 0.6M; beside the weight-
        # gradient convs the 4x4 layers' rendezvous waits for CUs and loses to the three kernels).
        self.bn_fused_max = int(os.environ.get("DPA_BN_FUSED_MAX", "2200000")) if dev.type == "cuda" else 0
        # (fp16 pairs: the data-gradient bound needs the whole tensor before the apply, which the
        # one-launch kernel's per-slice rendezvous cannot give -- the three-kernel backward runs)
        self.bn_fused_bwd_max = (int(os.environ.get("DPA_BN_FUSED_BWD_MAX", "600000"))
                                 if dev.type == "cuda" and self.np != 2 else 0)
        self.bn_fused_rmax = int(os.environ.get("DPA_BN_FUSED_RMAX", "64"))
        self._fgeo: Dict[tuple, bool] = {}
        fpart, fcnt = 0, 0
        if max(self.bn_fused_max, self.bn_fused_bwd_max) > 0 and hasattr(self.K, "bn_fused_geo"):
            for i, l in enumerate(L):
                for bwd in (False, True):
                    gq = self._fused_geo(i, N, bwd)
                    if gq is not None:
                        fpart, fcnt = max(fpart, gq[0]), max(fcnt, gq[1])
        self.fpart = torch.zeros(max(fpart, 1), **f32)
        self.fcnt = torch.zeros(max(fcnt, 32), dtype=torch.int32, device=dev)
        self.bn_tmo = torch.zeros(1, dtype=torch.int32, device=dev)
        # BN statistics from the forward conv's epilogue (conv_x3.hip epi_col_stats) for layers whose
        # conv runs one split and whose BN is not the one-launch kernel: the statistics pass's read
        # of z goes; DPA_EPI_STATS=0 keeps bn_stats_kernel
        self.epi_stats = (dev.type == "cuda" and os.environ.get("DPA_EPI_STATS", "1") == "1"
                          and hasattr(self.K, "conv_stats_rows"))
        epart = 0
        for i, l in enumerate(L):
            rows = self._epi_rows(i, N)
            if rows:
                epart = max(epart, 2 * ((N * l.hw * l.hw + rows - 1) // rows) * l.cout)
        self.epart = torch.empty(max(epart, 1), **f32)
        # BN reduction workspace
        self.part = torch.zeros(part_need, **f32)
        self.coef = torch.empty(4 * max(l.cout for l in L), **f32)  # [k1, c2, k3, mean] (bn.hip bwd_coef)
        self.loss_row = torch.zeros(N, **f32)
        self.dlogits = torch.zeros(N, num_classes, **f32)
        self.loss = torch.zeros(1, **f32)
        self.loss_accum = torch.zeros(1, **f32)
        self.correct = torch.zeros(N, dtype=torch.int32, device=dev)
        self.eval_acc = torch.zeros(2, **f32)
        self._eval_dirty = True
        self.health = (dev.type == "cuda" and hasattr(self.K, "health_copy")
                       and os.environ.get("DPA_STEP_HEALTH", "1") == "1")
        self._health_extra: List[tuple] = []
        self._health_ptrs = None
        self._health_out = None
        self._health_slot = 0
        self._health_pending = [False, False]
        self.init_parameters(seed=None)

    def _make_wgrad_stream(self, dev: torch.device):
        """The weight-gradient stream: a default-priority torch stream (a lowest-priority one was
        measured: no gain alone, and beside the RCCL comm stream the mixed queue priorities cost
        28 % of the step, docs/PERF_NOTES.md)."""
        return torch.cuda.Stream(dev)

    # ------------------------------------------------------------------ parameters / state
    @torch.no_grad()
    def init_parameters(self, seed: Optional[int] = None, module: Optional[torch.nn.Module] = None):
        """torch default init of the reference module (seeded like the reference: manual_seed
        before construction), copied into the arenas."""
        from .models.vgg import VGG

        if module is None:
            if seed is not None:
                torch.manual_seed(seed)
            module = VGG(self.spec.name, self.num_classes)
        self.load_state_dict(module.state_dict())

    @torch.no_grad()
    def load_state_dict(self, sd: Dict[str, torch.Tensor], strict: bool = True):
        sd = {k[7:] if k.startswith("module.") else k: v for k, v in sd.items()}
        seen = set()
        for l in self.spec.convs:
            w = sd[f"{l.conv_key}.weight"]  # OIHW
            dst = self.params[f"{l.conv_key}.weight"]
            dst.zero_()
            dst[..., :l.cin].copy_(w.permute(0, 2, 3, 1))
            for k in (f"{l.conv_key}.bias", f"{l.bn_key}.weight", f"{l.bn_key}.bias"):
                self.params[k].copy_(sd[k])
            for b in ("running_mean", "running_var"):
                self.buffers[f"{l.bn_key}.{b}"].copy_(sd[f"{l.bn_key}.{b}"])
            self.nbt[self.spec.convs.index(l)] = int(sd.get(f"{l.bn_key}.num_batches_tracked", torch.tensor(0)))
            seen |= {f"{l.conv_key}.weight", f"{l.conv_key}.bias", f"{l.bn_key}.weight", f"{l.bn_key}.bias",
                     f"{l.bn_key}.running_mean", f"{l.bn_key}.running_var", f"{l.bn_key}.num_batches_tracked"}
        for k in ("fc1.weight", "fc1.bias"):
            self.params[k].copy_(sd[k])
            seen.add(k)
        if strict:
            extra = set(sd) - seen
            if extra:
                raise KeyError(f"unexpected keys in state_dict: {sorted(extra)[:5]}")
        self._eval_dirty = True
        self.refresh_weight_planes()

    def refresh_weight_planes(self):
        """Re-split the parameter arena into the bf16 operand planes (one launch).  Needed after
        parameters change outside ``sgd_step`` (load, broadcast); the SGD kernel refreshes them
        itself."""
        if self.wplanes is not None:
            self.K.split_planes(self.params.flat, self.wplanes, self.h2_sw if self.np == 2 else 1.0)

    @torch.no_grad()
    def state_dict(self, prefix: str = "") -> "OrderedDict[str, torch.Tensor]":
        """Reference-layout state_dict (58 keys for VGG-11, OIHW fp32, CPU tensors)."""
        out: "OrderedDict[str, torch.Tensor]" = OrderedDict()
        for i, l in enumerate(self.spec.convs):
            out[prefix + f"{l.conv_key}.weight"] = (
                self.params[f"{l.conv_key}.weight"][..., :l.cin].permute(0, 3, 1, 2).contiguous().cpu())
            out[prefix + f"{l.conv_key}.bias"] = self.params[f"{l.conv_key}.bias"].cpu().clone()
            out[prefix + f"{l.bn_key}.weight"] = self.params[f"{l.bn_key}.weight"].cpu().clone()
            out[prefix + f"{l.bn_key}.bias"] = self.params[f"{l.bn_key}.bias"].cpu().clone()
            out[prefix + f"{l.bn_key}.running_mean"] = self.buffers[f"{l.bn_key}.running_mean"].cpu().clone()
            out[prefix + f"{l.bn_key}.running_var"] = self.buffers[f"{l.bn_key}.running_var"].cpu().clone()
            out[prefix + f"{l.bn_key}.num_batches_tracked"] = self.nbt[i].cpu().clone()
        out[prefix + "fc1.weight"] = self.params["fc1.weight"].cpu().clone()
        out[prefix + "fc1.bias"] = self.params["fc1.bias"].cpu().clone()
        return out

    def _to_torch_layout(self, name: str, t: torch.Tensor) -> torch.Tensor:
        if name.endswith(".weight") and t.dim() == 4:
            l = next(l for l in self.spec.convs if name == f"{l.conv_key}.weight")
            return t[..., :l.cin].permute(0, 3, 1, 2).contiguous()
        return t.clone()

    def _from_torch_layout(self, name: str, t: torch.Tensor, dst: torch.Tensor):
        if name.endswith(".weight") and dst.dim() == 4:
            l = next(l for l in self.spec.convs if name == f"{l.conv_key}.weight")
            dst.zero_()
            dst[..., :l.cin].copy_(t.permute(0, 2, 3, 1))
        else:
            dst.copy_(t)

    @torch.no_grad()
    def optimizer_state_dict(self) -> dict:
        """torch.optim.SGD-format state_dict (momentum buffers in OIHW)."""
        names = self.spec.param_names()
        state = {}
        if self.steps_taken > 0:
            for i, n in enumerate(names):
                state[i] = {"momentum_buffer": self._to_torch_layout(n, self.mom[n]).cpu()}
        return {"state": state,
                "param_groups": [{"lr": self.lr, "momentum": self.momentum, "dampening": 0,
                                  "weight_decay": self.weight_decay, "nesterov": False, "maximize": False,
                                  "foreach": None, "differentiable": False, "fused": None,
                                  "params": list(range(len(names)))}]}

    @torch.no_grad()
    def load_optimizer_state_dict(self, osd: dict):
        names = self.spec.param_names()
        pg = osd["param_groups"][0]
        self.lr, self.momentum, self.weight_decay = pg["lr"], pg["momentum"], pg["weight_decay"]
        st = osd.get("state", {})
        if st:
            for i, n in enumerate(names):
                self._from_torch_layout(n, st[i]["momentum_buffer"].to(self.device), self.mom[n])
            self.steps_taken = max(self.steps_taken, 1)
        else:
            self.mom.flat.zero_()
            self.steps_taken = 0

    def num_parameters(self) -> int:
        return sum(p.numel() for p in self.state_dict().values() if p.dtype == torch.float32) - sum(
            self.buffers.numels.values())

    def _fused_geo(self, i: int, n: int, bwd: bool):
        """(part_floats, cnt_words, blocks) when layer i's BN runs as one launch at batch n, else None."""
        lim = self.bn_fused_bwd_max if bwd else self.bn_fused_max
        if lim <= 0 or not hasattr(self.K, "bn_fused_geo"):
            return None
        l = self.spec.convs[i]
        if i == 0 or n * l.hw * l.hw * l.cout > lim:
            return None  # layer 0: conv0_fwd / bn_bwd_wgrad0 fuse its BN with the convolution instead
        ho = l.hw // 2 if l.pool else l.hw
        return self.K.bn_fused_geo(n * ho * ho, l.cout, l.pool, bwd, self.bn_fused_rmax)

    def _fused(self, i: int, n: int, bwd: bool) -> bool:
        key = (i, n, bwd)
        v = self._fgeo.get(key)
        if v is None:
            v = self._fgeo[key] = self._fused_geo(i, n, bwd) is not None
        return v

    # ------------------------------------------------------------------ kernel configs
    def _layer_impl(self, i: int) -> str:
        return self.impl if self.planes[i] else "fp32"

    def conv_config(self, i: int, kind: str, n: int):
        """(tile, effective splits, posmajor) for conv call `kind` of layer i at batch n: the measured
        table (tuning/mi355x.json) when it has the call, else the heuristic."""
        impl = self._layer_impl(i)
        l = self.spec.convs[i]
        key = (impl, kind, n, i)
        c = self._cfg_cache.get(key)
        if c is not None:
            return c
        M = n * l.hw * l.hw
        if kind == "fprop":
            gm, gn, gk = M, l.cout, 9 * l.cin_pad
        elif kind == "dgrad":
            gm, gn, gk = M, l.cin_pad, 9 * l.cout
        else:
            gm, gn, gk = M, l.cout, 9 * l.cin_pad
        t = tuning_table().get(conv_key(impl, kind, n, l.hw, l.cin_pad, l.cout))
        if t is None and impl == "h2":  # the fp16-pair kernels share x3's tiles: its measured plan
            t = tuning_table().get(conv_key("x3", kind, n, l.hw, l.cin_pad, l.cout))
        if t is not None:
            tile, s, pm = int(t[0]), int(t[1]), int(t[2])  # pm: bit 0 position-major, bit 1 column-tile order
        elif impl == "fp32":
            tile, s = conv_cfg("wgrad" if kind == "wgrad" else "fprop", gm, gn, gk)
            pm = l.hw <= 8
        else:  # bf16-plane kernels: 128x128/k32 tiles, ~512 blocks
            cd = lambda a_, b_: (a_ + b_ - 1) // b_
            tiles = cd(gn, 128) * cd(gk, 128) if kind == "wgrad" else cd(gm, 128) * cd(gn, 128)
            red = gm if kind == "wgrad" else gk
            tile, s = 0, max(1, min(128, _pow2_round(512 / max(tiles, 1))))
            while s > 1 and red // s < 64:
                s //= 2
            pm = l.hw <= 4
        if kind != "wgrad" or impl == "fp32":
            s = self.K.conv_splits(gm if kind == "wgrad" else gk, s) if impl == "fp32" else self.K.x3_splits(gk, s)
        else:
            s = self.K.x3_splits(gm, s)
        c = (tile, s, pm)
        self._cfg_cache[key] = c
        return c

    def _slab_need(self, i: int, kind: str, n: int) -> int:
        l = self.spec.convs[i]
        _, s, _ = self.conv_config(i, kind, n)
        if s <= 1:
            return 0
        M = n * l.hw * l.hw
        out = {"fprop": M * l.cout, "dgrad": M * l.cin_pad, "wgrad": l.cout * 9 * l.cin_pad}[kind]
        return s * out

    def conv_candidates(self, i: int, kind: str):
        impl = self._layer_impl(i)
        l = self.spec.convs[i]
        tiles = (0, 1) if impl == "fp32" else tuple(range(16))
        splits = (1, 2, 4, 8, 16, 32, 64, 128, 256, 512) if kind == "wgrad" else (1, 2, 4, 8, 16)
        pms = (0, 1) if impl == "fp32" else (0, 1, 2, 3)  # x3 tiles: bit 1 = column-tile-outer block order
        out = [(t, s, pm) for t in tiles for s in splits for pm in pms]
        if impl != "fp32":  # halo tiles ignore the row order flag
            if kind == "wgrad":
                ok = [t for t in HALO_WGRAD_TILES if halo_ok(kind, t, l.hw, l.cin_pad, l.cout)]
            else:
                cred, cout = (l.cin_pad, l.cout) if kind == "fprop" else (l.cout, l.cin_pad)
                np_ = {"x3": 3, "h2": 2}.get(impl, 1)
                ok = [t for t in HALO_TILES if halo_ok(kind, t, l.hw, cred, cout, np_)]
                ok += [t for t in POS_TILES if pos_ok(kind, t, l.hw, l.hw, cred, cout)]
            out += [(t, s, False) for t in ok for s in splits]
        return out

    def autotune(self, n: Optional[int] = None, iters: int = 3, verbose: bool = False,
                 only: Optional[List[str]] = None) -> Dict[str, list]:
        """Time every candidate (tile, splits, posmajor) of every conv call of the step at batch n on
        this GPU and adopt the fastest.  Returns {conv_key: [tile, splits, posmajor, ms]} (the
        format of tuning/mi355x.json).  Buffers must hold one step's data (run a step first).
        ``only``: tune just the calls whose conv_key contains one of these substrings."""
        n = n or self.max_batch
        res: Dict[str, list] = {}
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        L = self.spec.convs
        for i, l in enumerate(L):
            for kind in ("fprop", "dgrad", "wgrad"):
                if kind == "dgrad" and i == 0:
                    continue
                impl = self._layer_impl(i)
                key = (impl, kind, n, i)
                if only and not any(o in conv_key(impl, kind, n, l.hw, l.cin_pad, l.cout) for o in only):
                    continue
                best = None
                for cand in self.conv_candidates(i, kind):
                    tile, s, pm = cand
                    M = n * l.hw * l.hw
                    red = M if kind == "wgrad" else (9 * (l.cin_pad if kind == "fprop" else l.cout))
                    s = (self.K.conv_splits(red, s) if impl == "fp32" else self.K.x3_splits(red, s))
                    self._cfg_cache[key] = (tile, s, pm)
                    if self._slab_need(i, kind, n) * 4 > (256 << 20):
                        continue  # split-K workspace beyond 256 MiB: not a sensible plan
                    fn = {"fprop": lambda: self._conv_fwd(i, self.x0[:n], n, reduce=False),
                          "dgrad": lambda: self._conv_dgrad(i, n),
                          "wgrad": lambda: self._conv_wgrad(i, self.x0[:n], n)}[kind]
                    fn()
                    ev0.record()
                    for _ in range(iters):
                        fn()
                    ev1.record()
                    torch.cuda.synchronize(self.device)
                    ms = ev0.elapsed_time(ev1) / iters
                    if best is None or ms < best[3]:
                        best = [tile, s, pm, ms]
                self._cfg_cache[key] = tuple(best[:3])
                ck = conv_key(impl, kind, n, l.hw, l.cin_pad, l.cout)
                res[ck] = best
                if verbose:
                    print(ck, best, flush=True)
        return res

    def _ensure_slab(self, numel: int, wgrad: bool = False):
        if wgrad and self.wslab is not None:
            if numel > self.wslab.numel():
                self.wslab = torch.empty(numel, device=self.device, dtype=torch.float32)
        elif numel > self.slab.numel():
            self.slab = torch.empty(numel, device=self.device, dtype=torch.float32)

    def _in_planes(self, i: int, n: int) -> torch.Tensor:
        return self.x0p[:, :n] if i == 0 else self.a3[i - 1][:, :n]

    def _epi_rows(self, i: int, n: int) -> int:
        """Rows per statistics partial when layer i's BN takes its statistics from the conv
        epilogue at batch n, else 0."""
        if not (self.epi_stats and self.planes[i] and i > 0) or self._fused(i, n, False):
            return 0
        tile, s, _ = self.conv_config(i, "fprop", n)
        return self.K.conv_stats_rows(tile) if s == 1 else 0

    def _conv_fwd(self, i: int, x: torch.Tensor, n: int, reduce: bool, stats: Optional[torch.Tensor] = None) -> int:
        """Forward conv of layer i into z[i] (or split-K slabs); returns the split count left
        UNREDUCED in self.slab (1 = result is in z[i]).  stats: BN partials from the epilogue."""
        l = self.spec.convs[i]
        tile, s, pm = self.conv_config(i, "fprop", n)
        self._ensure_slab(self._slab_need(i, "fprop", n))
        z = self.z[i][:n]
        slab = self.slab if s > 1 else None
        if self.planes[i]:
            self.K.conv_x3_fprop(self._in_planes(i, n), self.w3[i], z, slab, 1, 1, s, tile, reduce, pm, stats,
                                 **self._h2(1.0 / (self.h2_sa * self.h2_sw)))
        else:
            xin = x if i == 0 else self.a[i - 1][:n]
            self.K.conv_fprop(xin, self.params[f"{l.conv_key}.weight"], z, slab, 1, 1, s, tile, False, reduce, pm)
        return 1 if (reduce or s == 1) else s

    def _conv_dgrad(self, i: int, n: int, sig_val: int = 0) -> int:
        """Data gradient of layer i into g[i-1] (or slabs); returns the unreduced split count.
        ``sig_val`` > 0: the kernel stores it into ksig[i] when it starts (plane convs only)."""
        l = self.spec.convs[i]
        tile, s, pm = self.conv_config(i, "dgrad", n)
        self._ensure_slab(self._slab_need(i, "dgrad", n))
        slab = self.slab if s > 1 else None
        out = self.g[i - 1][:n]
        if self.planes[i]:
            h2 = self._h2(1.0 / self.h2_sw, i)
            if sig_val > 0:
                self.K.conv_x3_dgrad(self.dz3[i][:, :n], self.w3[i], out, slab, 1, 1, s, tile, False, pm,
                                     sig=self.ksig[i:i + 1], sig_val=sig_val, **h2)
            else:
                self.K.conv_x3_dgrad(self.dz3[i][:, :n], self.w3[i], out, slab, 1, 1, s, tile, False, pm, **h2)
        else:
            self.K.conv_fprop(self.dz[i][:n], self.params[f"{l.conv_key}.weight"], out, slab, 1, 1, s, tile, True,
                              False, pm)
        return s

    def _wgrad_on_side(self, i: int) -> bool:
        """Whether layer i's weight gradient runs on the wgrad stream (every layer but the first)."""
        return self.wstream is not None and i > 0

    def _conv_wgrad(self, i: int, x: torch.Tensor, n: int):
        l = self.spec.convs[i]
        tile, s, pm = self.conv_config(i, "wgrad", n)
        side = self._wgrad_on_side(i)
        self._ensure_slab(self._slab_need(i, "wgrad", n), wgrad=side)
        slab = (self.wslab if side else self.slab) if s > 1 else None
        dw = self.grads[f"{l.conv_key}.weight"]
        if self.planes[i]:
            self.K.conv_x3_wgrad(self._in_planes(i, n), self.dz3[i][:, :n], dw, slab, 1, 1, s, tile, pm,
                                 **self._h2(1.0 / self.h2_sa, i))
        else:
            xin = x if i == 0 else self.a[i - 1][:n]
            self.K.conv_wgrad(xin, self.dz[i][:n], dw, slab, 1, 1, s, tile, pm)

    def _h2(self, oscale: float, dz_layer: Optional[int] = None) -> dict:
        """fp16-pair conv keywords: the output scale 1 / (s_a s_b) of the constant scales, and the
        bound word of layer ``dz_layer``'s data gradient when dz is an operand (empty otherwise)."""
        if self.np != 2:
            return {}
        kw = {"oscale": oscale}
        if dz_layer is not None:
            kw["obound"] = self.dzb[dz_layer:dz_layer + 1]
        return kw

    def _act_out(self, i: int, n: int) -> torch.Tensor:
        """Where bn_apply of layer i writes: bf16 planes if layer i+1 consumes planes, else fp32."""
        return self.a3[i][:, :n] if self.a3[i] is not None else self.a[i][:n]

    # ------------------------------------------------------------------ training step
    def forward_backward(self, x: torch.Tensor, target: torch.Tensor,
                         grad_ready: Optional[Callable[[List[str]], None]] = None,
                         pre_forward: Optional[Callable[[], None]] = None,
                         params_free: Optional[Callable[[List[str]], None]] = None) -> torch.Tensor:
        """One training forward+backward on x [n,H,W,4] (NHWC fp32, 4th channel zero).
        Gradients land in ``self.grads``; the batch-mean loss in ``self.loss`` (device) and is
        also accumulated into ``self.loss_accum``.  Returns ``self.loss``.

        Callbacks (the gradient-sync strategy's hooks):
          ``grad_ready(names)``  every kernel writing those gradients has been enqueued; called with
                                 the stream that ran the last of them current (wgrad stream or main);
          ``params_free(names, signal=None)`` every kernel of this step READING those parameters
                                 (or their bf16 planes) has been enqueued; called with the main
                                 stream current.  ``signal`` (when not None): a (flag, value) pair
                                 that a LATER main-stream kernel raises when it starts — waiting for
                                 it (``wait_signal``) orders after those readers without a queue
                                 marker on the main stream.
        Once both have fired for a tensor its optimizer step may run while backward continues."""
        K, P, G = self.K, self.params, self.grads
        n = x.shape[0]
        L = self.spec.convs
        buffers_wait = pre_forward() if pre_forward is not None else None
        epoch = 0
        if self.ksignal and not torch.cuda.is_current_stream_capturing():
            self._sig_epoch += 1
            epoch = self._sig_epoch
        if self.x0p is not None and not (self.fused_conv0 and self.fused_wgrad0):  # plane kernels read x0p
            K.pad_split8(x, self.x0p[:, :n])
        for i, l in enumerate(L):
            z, st = self.z[i][:n], self.stats[i]
            if i == 0 and self.fused_conv0:
                if buffers_wait is not None:
                    buffers_wait()
                    buffers_wait = None
                K.conv0_fwd(x, P[f"{l.conv_key}.weight"], z, self.part0, P[f"{l.bn_key}.weight"],
                            P[f"{l.bn_key}.bias"], P[f"{l.conv_key}.bias"], self.buffers[f"{l.bn_key}.running_mean"],
                            self.buffers[f"{l.bn_key}.running_var"], self.nbt[i:i + 1], st["mean"], st["invstd"],
                            st["scale"], st["shift"], self.bn_momentum, self.bn_eps)
                K.bn_apply(z, self._act_out(i, n), st["scale"], st["shift"], l.pool)
                continue
            erows = self._epi_rows(i, n)
            if erows and self.epart.numel() < 2 * ((n * l.hw * l.hw + erows - 1) // erows) * l.cout:
                # a conv plan changed after construction (tools/tune_step.py): more partial rows
                self.epart = torch.empty(2 * ((n * l.hw * l.hw + erows - 1) // erows) * l.cout,
                                         dtype=torch.float32, device=self.device)
            ns = self._conv_fwd(i, x, n, reduce=False, stats=self.epart if erows else None)
            if buffers_wait is not None:  # BN buffers (being broadcast) are first touched here
                buffers_wait()
                buffers_wait = None
            if erows:
                M = n * l.hw * l.hw
                K.bn_finalize(self.epart, (M + erows - 1) // erows, erows, M, P[f"{l.bn_key}.weight"],
                              P[f"{l.bn_key}.bias"], P[f"{l.conv_key}.bias"],
                              self.buffers[f"{l.bn_key}.running_mean"], self.buffers[f"{l.bn_key}.running_var"],
                              self.nbt[i:i + 1], st["mean"], st["invstd"], st["scale"], st["shift"],
                              self.bn_momentum, self.bn_eps)
                if not (i == len(L) - 1 and self.fused_head):
                    K.bn_apply(z, self._act_out(i, n), st["scale"], st["shift"], l.pool)
                continue
            if self._fused(i, n, False):
                # the head kernel applies it: statistics and coefficients only
                head = i == len(L) - 1 and self.fused_head
                K.bn_fused_fwd(self.slab if ns > 1 else z, ns, z, l.pool, self.bn_fused_rmax, self.fpart, self.fcnt,
                               P[f"{l.bn_key}.weight"], P[f"{l.bn_key}.bias"], P[f"{l.conv_key}.bias"],
                               self.buffers[f"{l.bn_key}.running_mean"], self.buffers[f"{l.bn_key}.running_var"],
                               self.nbt[i:i + 1], st["mean"], st["invstd"], st["scale"], st["shift"],
                               None if head else self._act_out(i, n), self.bn_momentum, self.bn_eps, self.bn_tmo,
                               self.bn_fused_timeout_us)
                continue
            K.bn_fwd_stats(self.slab if ns > 1 else z, ns, z, self.part, P[f"{l.bn_key}.weight"],
                           P[f"{l.bn_key}.bias"], P[f"{l.conv_key}.bias"],
                           self.buffers[f"{l.bn_key}.running_mean"], self.buffers[f"{l.bn_key}.running_var"],
                           self.nbt[i:i + 1], st["mean"], st["invstd"], st["scale"], st["shift"], self.bn_momentum,
                           self.bn_eps)
            if i == len(L) - 1 and self.fused_head:
                continue  # applied inside the head kernel below
            K.bn_apply(z, self._act_out(i, n), st["scale"], st["shift"], l.pool)
        feat = self.a[-1][:n].view(n, -1)
        bn_in = (dict(bn_z=self.z[-1][:n], bn_scale=self.stats[-1]["scale"], bn_shift=self.stats[-1]["shift"])
                 if self.fused_head else {})
        # the head's weight gradient / batch loss kernel goes to the wgrad stream (nothing on the critical
        # path reads them); it waits for the first BN backward's start signal, which implies the row
        # kernel (features, dlogits) has completed.
        head_side = bool(epoch) and self.wstream is not None and self.head_side
        head_args = (feat, P["fc1.weight"], P["fc1.bias"], target, self.loss_row[:n], self.dlogits[:n],
                     self.g[-1][:n].view(n, -1), G["fc1.weight"], G["fc1.bias"], self.loss, self.loss_accum)
        K.fc_ce_train(*head_args, **bn_in, **({"parts": 1} if head_side else {}))
        if grad_ready is not None and not head_side:
            grad_ready(["fc1.weight", "fc1.bias"])
        # Kernel-start signals (epoch > 0, signal.hip): each BN backward raises bsig[i] when it starts,
        # so every main-stream kernel enqueued before it (the data-gradient conv of layer i+1, the
        # head) has completed.  params_free is therefore reported AFTER the next BN backward is
        # enqueued, with its signal: the sync's update waits on it instead of an event recorded on
        # the main stream.  Likewise layer i+1's wgrad-stream work (wait for dgrad(i+1)'s start
        # signal, wgrad, grad_ready) is enqueued after bn_bwd(i).  A wait is thus always enqueued
        # after the kernel that raises its signal: it completes even if streams share a hardware
        # queue.
        sigs = bool(epoch) and self.free_signal
        free_later: List[List[str]] = []  # params_free calls waiting for the next BN backward
        side_later: Optional[tuple] = None  # (layer, names) whose wgrad-stream work is deferred
        if params_free is not None:
            if sigs:
                free_later.append(["fc1.weight", "fc1.bias"])
            else:
                params_free(["fc1.weight", "fc1.bias"])
        gsplit = 1  # split-K slabs of g[i] left unreduced by the previous dgrad (summed inside bn_bwd)
        ws = self.wstream
        main = torch.cuda.current_stream(self.device) if ws is not None else None

        def side_work(j: int, nm: List[str]):
            with torch.cuda.stream(ws):
                K.wait_signal(self.ksig[j:j + 1], epoch, self.ksig_timeout_us, self.ksig_tmo)
                self._conv_wgrad(j, x, n)
                if grad_ready is not None:
                    grad_ready(nm)

        joined = False

        def drain_side():
            """Before layer 0's gradients are reported from the main stream: layer 0 shares the last
            bucket with layer 1, whose weight gradient runs on the wgrad stream, and the bucket's
            collective is ordered after the stream that reports last.  Make the main stream wait
            for the wgrad stream first (the end-of-backward join, moved up), so the collective sees
            every producer of the bucket."""
            nonlocal joined, side_later
            if ws is None or joined:
                return
            if side_later is not None:
                side_work(*side_later)
                side_later = None
            self._end_join(main, ws, epoch)
            joined = True

        def after_bn(i: int):
            nonlocal free_later, side_later, head_side
            if head_side:  # first BN backward enqueued: its start signal orders the head's weight gradient
                with torch.cuda.stream(ws):
                    K.wait_signal(self.bsig[i:i + 1], epoch, self.ksig_timeout_us, self.ksig_tmo)
                    K.fc_ce_train(*head_args, parts=2)
                    if grad_ready is not None:
                        grad_ready(["fc1.weight", "fc1.bias"])
                head_side = False
            for nm in free_later:
                params_free(nm, signal=(self.bsig[i:i + 1], epoch))
            free_later = []
            if side_later is not None:
                side_work(*side_later)
                side_later = None

        for i in range(len(L) - 1, -1, -1):
            l = L[i]
            st = self.stats[i]
            z = self.z[i][:n]
            g = self.g[i][:n]
            dzbuf = self.dz3[i][:, :n] if self.planes[i] else self.dz[i][:n]
            names = [f"{l.conv_key}.weight", f"{l.conv_key}.bias", f"{l.bn_key}.weight", f"{l.bn_key}.bias"]
            bsig = dict(sig=self.bsig[i:i + 1], sig_val=epoch) if epoch else {}
            if i == 0 and self.fused_wgrad0:
                K.bn_bwd_wgrad0(self.slab if gsplit > 1 else g, gsplit, g, z, st["scale"], st["shift"], st["mean"],
                                st["invstd"], P[f"{l.bn_key}.weight"], self.part, self.coef, G[f"{l.bn_key}.weight"],
                                G[f"{l.bn_key}.bias"], G[f"{l.conv_key}.bias"], x, self.wpart,
                                G[f"{l.conv_key}.weight"], **bsig)
                after_bn(i)
                drain_side()
                if grad_ready is not None:
                    grad_ready(names)
                if params_free is not None:
                    params_free(names)
                continue
            if self._fused(i, n, True):
                K.bn_fused_bwd(self.slab if gsplit > 1 else g, gsplit, z, l.pool, self.bn_fused_rmax, self.fpart,
                               self.fcnt, st["scale"], st["shift"], st["mean"], st["invstd"], P[f"{l.bn_key}.weight"],
                               G[f"{l.bn_key}.weight"], G[f"{l.bn_key}.bias"], G[f"{l.conv_key}.bias"], dzbuf,
                               self.bn_tmo, self.bn_fused_timeout_us, **bsig)
            else:
                bnd = {"bound": self.dzb[i:i + 1]} if self.np == 2 and self.planes[i] else {}
                K.bn_bwd(self.slab if gsplit > 1 else g, gsplit, g, z, st["scale"], st["shift"], st["mean"],
                         st["invstd"], P[f"{l.bn_key}.weight"], self.part, self.coef, G[f"{l.bn_key}.weight"],
                         G[f"{l.bn_key}.bias"], G[f"{l.conv_key}.bias"], dzbuf, l.pool, **bsig, **bnd)
            after_bn(i)
            if not self._wgrad_on_side(i):
                # wgrad first: it needs no slab that bn_bwd(i-1) reads, and its bucket becomes ready early.
                # Layer 0's wgrad has nothing left to overlap with, so it stays on the main stream (a
                # stream hop costs ~15 us on MI355X, tools/event_overhead.py)
                self._conv_wgrad(i, x, n)
                if i == 0:
                    drain_side()
                if grad_ready is not None:
                    grad_ready(names)
                if i > 0:
                    gsplit = self._conv_dgrad(i, n)
                if params_free is not None:  # dgrad(i) was the last reader of layer i's weights
                    if sigs and i > 0:
                        free_later.append(names)
                    else:
                        params_free(names)
                continue
            # two streams: the critical path (dgrad -> BN backward of layer i-1) is issued first on
            # the main stream; wgrad(i) follows bn_bwd(i) on the wgrad stream, and the bucket's
            # collective is ordered after it (the comm region waits on the stream current here)
            if epoch and self.planes[i]:
                # no queue marker on the main stream: dgrad(i) signals its own start, which implies
                # bn_bwd(i) (dz) has completed; the wgrad stream polls for it (signal.hip)
                gsplit = self._conv_dgrad(i, n, sig_val=epoch)
                if params_free is not None:
                    if sigs:
                        free_later.append(names)
                    else:
                        params_free(names)
                if sigs:
                    side_later = (i, names)
                else:
                    side_work(i, names)
                continue
            ev = self._wev[i]
            ev.record(main)
            if i > 0:
                gsplit = self._conv_dgrad(i, n)
            if params_free is not None:
                if sigs:
                    free_later.append(names)
                else:
                    params_free(names)
            ev.wait(ws)
            with torch.cuda.stream(ws):
                self._conv_wgrad(i, x, n)
                if grad_ready is not None:
                    grad_ready(names)
        for nm in free_later:  # no BN backward left to carry a signal
            params_free(nm)
        if side_later is not None:
            side_work(*side_later)
        if ws is not None and not joined:
            self._end_join(main, ws, epoch)
        self._eval_dirty = True
        return self.loss

    def _end_join(self, main, ws, epoch: int):
        """The main stream waits for everything queued so far on the wgrad stream."""
        if self.jsig is None or not epoch:
            self._join(main, ws)
            return
        with torch.cuda.stream(ws):
            self.K.set_signal(self.jsig, epoch)
        self.K.wait_signal(self.jsig, epoch, self.ksig_timeout_us, self.ksig_tmo)

    def sgd_step(self, grad_scale: float = 1.0, offset: int = 0, count: int = -1, first: Optional[bool] = None):
        """Fused SGD over the arena (or the [offset, offset+count) slice of it)."""
        self._sgd(grad_scale, offset, count, self.steps_taken == 0 if first is None else first)

    def _sgd(self, grad_scale: float, offset: int, count: int, first: bool):
        self.K.sgd_flat(self.params.flat, self.grads.flat, self.mom.flat, self.lr, self.momentum, self.weight_decay,
                        grad_scale, first, offset, count, self.wplanes)

    def wait_signal(self, signal):
        """The current stream waits (one polling wave, bounded) for a ``(flag, value)`` signal."""
        self.K.wait_signal(signal[0], signal[1], self.ksig_timeout_us, self.ksig_tmo)

    def check_signals(self):
        """Raise if a wgrad-stream wait gave up (its producer's signal never arrived: the weight
        gradients of that step were computed from an unfinished BN backward).  Synchronises."""
        self.health_flush()
        if self.ksig_tmo is not None and int(self.ksig_tmo.item()) != 0:
            raise RuntimeError("VGGEngine: a wgrad-stream signal wait timed out "
                               f"(DPA_KSIGNAL_TIMEOUT_US={self.ksig_timeout_us}); weight gradients are invalid")
        if self.np == 2 and self.K.h2_overflow(True):
            raise RuntimeError("VGGEngine: an fp16-pair operand split left float16's range (a weight beyond "
                               f"{65504 / self.h2_sw:g} or an activation beyond {65504 / self.h2_sa:g}); "
                               "this step's convolutions are invalid")
        if int(self.bn_tmo.item()) != 0:
            raise RuntimeError("VGGEngine: a one-launch BatchNorm slice rendezvous timed out "
                               f"(DPA_BN_FUSED_TIMEOUT_US={self.bn_fused_timeout_us}); this step's "
                               "activations / gradients are invalid")

    def finish_step(self):
        self.steps_taken += 1
        self._eval_dirty = True
        self.health_mark()

    # ------------------------------------------------------------------ per-step health
    # Every step ends with a one-wave kernel (signal.hip health_kernel) that copies the device-side
    # error words -- the fp16-pair overflow words of every kernel file, the wgrad-stream wait
    # timeout, the one-launch BN rendezvous timeout, and any word a communicator registered
    # (add_health_word: the peer-collective timeout) -- into one of two pinned host slots.  After
    # enqueueing step k the host reads step k-1's slot (its event: by then the GPU is working on
    # step k, so the host stays one step ahead and the device never idles) and raises if any word
    # is set: a step that went wrong stops the run at the next step, before its parameters are
    # used for more than one further step or saved.  DPA_STEP_HEALTH=0 turns it off.
    def add_health_word(self, name: str, addr: int):
        """Register one more device int word (by address) for the per-step health snapshot."""
        if all(a != int(addr) for _, a in self._health_extra):
            self._health_extra.append((name, int(addr)))
            self._health_ptrs = None

    def _health_setup(self):
        names, addrs = [], []
        if self.np == 2:
            for nm, a in zip(("conv", "bn", "sgd", "bn_fused"), self.K.h2_overflow_addrs()):
                names.append(f"fp16-pair overflow ({nm} kernels)")
                addrs.append(a)
        if self.ksig_tmo is not None:
            names.append("wgrad-stream signal wait timeout")
            addrs.append(self.ksig_tmo.data_ptr())
        names.append("one-launch BatchNorm rendezvous timeout")
        addrs.append(self.bn_tmo.data_ptr())
        for nm, a in self._health_extra:
            names.append(nm)
            addrs.append(a)
        self._health_names = names
        self._health_ptrs = torch.tensor(addrs, dtype=torch.int64, device=self.device)
        if self._health_out is None:
            self._health_out = [torch.zeros(64, dtype=torch.int32).pin_memory() for _ in range(2)]
            self._health_ev = [torch.cuda.Event() for _ in range(2)]

    def health_mark(self):
        """Snapshot this step's error words (async) and check the previous step's snapshot."""
        if not self.health or torch.cuda.is_current_stream_capturing():
            return
        if self._health_ptrs is None:
            self._health_setup()
        k = self._health_slot
        self._health_slot ^= 1
        self.K.health_copy(self._health_ptrs, self._health_out[k], self.steps_taken)
        self._health_ev[k].record()
        self._health_pending[k] = True
        self._health_check(k ^ 1)

    def _health_check(self, j: int):
        if not self._health_pending[j]:
            return
        self._health_ev[j].synchronize()
        self._health_pending[j] = False
        v = self._health_out[j].tolist()
        bad = [nm for nm, x in zip(self._health_names, v) if x != 0]
        if bad:
            raise RuntimeError(f"VGGEngine: step {v[63]} failed its health check: {', '.join(bad)} "
                               "(that step's results are invalid; the run stops here)")

    def health_flush(self):
        """Check every snapshot still pending (synchronises with the last marked step)."""
        if self.health and self._health_ptrs is not None:
            for j in (self._health_slot ^ 1, self._health_slot):
                self._health_check(j)

    # ------------------------------------------------------------------ evaluation
    def begin_eval(self):
        for i, l in enumerate(self.spec.convs):
            self.K.bn_eval_params(self.params[f"{l.bn_key}.weight"], self.params[f"{l.bn_key}.bias"],
                                  self.params[f"{l.conv_key}.bias"], self.buffers[f"{l.bn_key}.running_mean"],
                                  self.buffers[f"{l.bn_key}.running_var"], self.eval_ss[i]["scale"],
                                  self.eval_ss[i]["shift"], self.bn_eps)
        self.eval_acc.zero_()
        self._eval_dirty = False

    def eval_batch(self, x: torch.Tensor, target: torch.Tensor, logits: Optional[torch.Tensor] = None):
        """Eval-mode forward (running stats); accumulates [sum of batch-mean losses, #correct]
        into ``self.eval_acc``."""
        if self._eval_dirty:
            raise RuntimeError("call begin_eval() after the last parameter update")
        n = x.shape[0]
        P = self.params
        if self.x0p is not None and not self.fused_conv0:
            self.K.pad_split8(x, self.x0p[:, :n])
        for i, l in enumerate(self.spec.convs):
            if i == 0 and self.fused_conv0:
                self.K.conv0_fwd(x, P[f"{l.conv_key}.weight"], self.z[0][:n])
            else:
                self._conv_fwd(i, x, n, reduce=True)
            self.K.bn_apply(self.z[i][:n], self._act_out(i, n), self.eval_ss[i]["scale"], self.eval_ss[i]["shift"],
                            l.pool)
        inp = self.a[-1][:n]
        self.K.fc_ce_eval(inp.view(n, -1), P["fc1.weight"], P["fc1.bias"], target, self.loss_row[:n],
                          self.correct[:n], logits, self.eval_acc)
        return self.eval_acc
