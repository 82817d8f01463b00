"""Batched DQN self-play driver on the device env (SURVEY.md section 8 row f-1,
BASELINE.json configs[3]: batch 65,536 with the legal-action mask and the
198-float observation feeding the reference trainer's DQN).

The reference trainer (train_deepq_pytorch.py) plays ONE env on the host:
per step it rolls dice, lists moves, runs DQNAgent.act over Python lists of
(move1, move2) combinations (:411-600), steps the env, shapes the reward
(:885-908), stores the transition and trains on a 64-sample prioritized
minibatch (:279-342, :602-750).  Here every piece works on B envs at once
without leaving the GPU:

  observation   VecNardeEnv.tesauro198()  (k_observe, README.md:42-102) or
                the reference's int32[24] perspective board (state_size 24)
  move-1 mask   VecNardeEnv.legal_mask()        (k_mask576: exactly the codes
                                                 NardeEnv.step accepts)
  move-2 mask   VecNardeEnv.legal_mask_move2()  (k_mask576_move2: the codes
                step accepts after the chosen move 1 -- the reference's act()
                guesses them from the pre-move board, :452-503)
                (greedy="reference": act()'s own candidate sets instead,
                VecNardeEnv.act_masks, k_act_masks)
  Q-values      DecomposedDQN, the reference's architecture and parameter
                names (:184-277), so its checkpoints load; move-2 Q-values
                use the column-gather identity below instead of a one-hot
                concat GEMM
  policy        masked epsilon-greedy; explore="plays": random.choice over
                act()'s (move1, move2) combinations (k_explore_plays, :514-515)
  env step      VecNardeEnv.step(actions)  (k_step, auto-reset)
  replay        DeviceReplay: prioritized replay with the reference's
                alpha/beta/epsilon rules on device tensors (:279-342)
  update        the reference's decomposed double-head DQN loss (:653-720),
                Adam, grad-norm clip 10, target sync every 10 updates,
                epsilon decay per update

move2_head(cat(features, onehot(m1))) = features @ Wf^T + Wm[:, m1] + b with
W = [Wf | Wm]: mathematically identical to the reference's one-hot concat,
equal in fp32 up to summation order (tests/test_dqn_cpu.py).
"""
import ctypes
import os

import torch
import torch.nn as nn

from . import _lib

MOVES = 576


class DecomposedDQN(nn.Module):
    """train_deepq_pytorch.py:184-222 (same layers, same parameter names)."""

    def __init__(self, state_size, move_space_size=MOVES):
        super().__init__()
        self.move_space_size = move_space_size
        self.feature_network = nn.Sequential(
            nn.Linear(state_size, 256), nn.ReLU(), nn.Linear(256, 256), nn.ReLU())
        self.move1_head = nn.Linear(256, move_space_size)
        self.move2_head = nn.Linear(256 + move_space_size, move_space_size)

    def features(self, x):
        return self.feature_network(x)

    def features_nograd(self, x):
        """features() for inference: bias + ReLU in the GEMM epilogue
        (torch._addmm_activation -> hipBLASLt), bit-equal to the module path
        at these shapes and ~50 us cheaper per 65,536 rows; no autograd."""
        l1, l2 = self.feature_network[0], self.feature_network[2]
        h = torch._addmm_activation(l1.bias, x, l1.weight.t())
        return torch._addmm_activation(l2.bias, h, l2.weight.t())

    def move2_from_features(self, f, move1):
        """move2 Q-values given move-1 codes, without materialising the
        one-hot concat: W[:, :256] f + W[:, 256 + m1] + b."""
        w = self.move2_head.weight
        out = torch.nn.functional.linear(f, w[:, :256], self.move2_head.bias)
        return out + w[:, 256:].t().index_select(0, move1)

    def forward(self, x, selected_move1=None):
        f = self.features(x)
        if selected_move1 is None:
            return self.move1_head(f)
        return self.move2_from_features(f, selected_move1)


def expand_mask(mask576):
    """(B,9) int64 bit masks -> (B,576) bool."""
    shifts = torch.arange(64, device=mask576.device, dtype=torch.int64)
    bits = (mask576.unsqueeze(-1) >> shifts) & 1
    return bits.view(mask576.shape[0], MOVES).bool()


def nearest_positive(p, idx):
    """A sampled row never has priority 0 (a pending row: its weight would be
    inf and the batch's weights NaN): where p[idx] == 0 take the last row
    before idx with p > 0, else the first one after it -- k_per_sample's
    rule.  Only a rounded-up u * total (the clamp to n - 1) or a prefix sum
    whose flat run steps by an ulp can pick such a row."""
    bad = ~(p[idx] > 0)  # (no host-side early exit: graph-capturable)
    n = p.shape[0]
    ar = torch.arange(n, device=p.device)
    pos = p > 0
    last = torch.where(pos, ar, torch.full_like(ar, -1)).cummax(0).values  # last positive <= i
    nxt = torch.where(pos, ar, torch.full_like(ar, n)).flip(0).cummin(0).values.flip(0)  # first >= i
    before = last[(idx - 1).clamp(min=0)]
    before = torch.where(idx > 0, before, torch.full_like(before, -1))
    after = nxt[(idx + 1).clamp(max=n - 1)]
    after = torch.where(idx < n - 1, after, torch.full_like(after, n))
    fix = torch.where(before >= 0, before, torch.where(after < n, after, idx))
    return torch.where(bad, fix, idx)


def masked_argmax(scores, mask):
    """argmax over legal entries; 0 where nothing is legal (the reference's
    'no move' code, train_deepq_pytorch.py:504-505).  Torch reference of
    policy_576's greedy half."""
    neg = torch.finfo(scores.dtype).min
    best = scores.masked_fill(~mask, neg).argmax(1)
    return torch.where(mask.any(1), best, torch.zeros_like(best))


def policy_576(q, mask576, epsilon, seed, tag, head, out=None, add=None):
    """Masked epsilon-greedy codes (B,) int64 from Q-values (B,576) f32 and
    the env's (B,9) bit masks: one HIP kernel (k_policy576), no (B,576)
    intermediates.  Same tag for both heads of a step = one shared explore
    decision per env.  epsilon / tag may be Python numbers or device scalars
    (f32 / int64 0-d tensors, read by the kernel at run time: graph-safe).
    add = (table (576,576) f32, rows (B,) int64): greedy values become
    q[i] + table[rows[i]] (one fp32 add, fused).  Greedy picks follow
    torch.argmax over the legal codes: the first maximum, a NaN Q-value
    beating every number (the first NaN); a legal code is always returned."""
    q = q.contiguous()
    if q.dtype != torch.float32 or q.shape[1] != MOVES:
        raise ValueError("q must be (B, 576) float32")
    if out is None:
        out = torch.empty(q.shape[0], dtype=torch.int64, device=q.device)
    stream = ctypes.c_void_p(torch.cuda.current_stream(q.device).cuda_stream)
    lib = _lib.load()
    args = (q.device.index, _lib.ptr(q), q.stride(0), _lib.ptr(mask576.contiguous()), q.shape[0])
    if torch.is_tensor(epsilon) or torch.is_tensor(tag) or add is not None:
        eps = torch.as_tensor(epsilon, dtype=torch.float32, device=q.device)
        tg = torch.as_tensor(tag, dtype=torch.int64, device=q.device)
        tab, rows, ld = None, None, 0
        if add is not None:
            tab, rows = add
            if (tab.dtype != torch.float32 or tab.dim() != 2 or tuple(tab.shape) != (MOVES, MOVES)
                    or tab.stride(1) != 1):
                raise ValueError("add table must be (576, 576) float32 with unit column stride "
                                 "(one row per move-1 code; the kernel keeps row indices in 0..575)")
            rows = rows.to(torch.int64).contiguous()
            if rows.shape != (q.shape[0],):
                raise ValueError("add rows must be (B,)")
            ld = tab.stride(0)
        _lib.check(lib.narde_policy_masked_argmax576_dev(
            *args, _lib.ptr(eps), int(seed) & (2 ** 64 - 1), _lib.ptr(tg), int(head), _lib.ptr(tab), ld,
            _lib.ptr(rows), _lib.ptr(out), stream), "narde_policy_masked_argmax576_dev")
        return out
    _lib.check(lib.narde_policy_masked_argmax576(
        *args, float(epsilon), int(seed) & (2 ** 64 - 1), int(tag) & 0xFFFFFFFF, int(head), _lib.ptr(out),
        stream), "narde_policy_masked_argmax576")
    return out


def head_policy_576(f, weight, bias, mask576, epsilon, seed, tag, head, out=None, move1=None, out16=None):
    """policy_576 with the head fused in (k_head_policy576): the Q-value of
    each legal code only, q_c = f . weight[c, :256] + bias[c] (+ weight[c,
    256 + move1] when move1 (B,) is given: the move-2 head's one-hot
    column), then the masked argmax / exploration of policy_576 (the same
    draws).  f (B,256) f32, weight (576, >=256) f32 with 16-B aligned rows;
    epsilon / tag: device scalars or numbers (device scalars: graph-safe).
    Replaces a dense (B,256)x(256,576) GEMM per head; greedy picks may
    differ from the dense head's only between codes whose Q-values tie to
    fp32 rounding."""
    if f.dtype != torch.float32 or f.dim() != 2 or f.shape[1] != 256 or f.stride(1) != 1:
        raise ValueError("f must be (B, 256) float32 with unit column stride")
    if weight.dtype != torch.float32 or weight.shape[0] != MOVES or weight.stride(1) != 1 or weight.shape[1] < 256:
        raise ValueError("weight must be (576, >=256) float32 with unit column stride")
    if move1 is not None and weight.shape[1] < 256 + MOVES:
        raise ValueError("the one-hot column needs the move-2 head's (576, 256 + 576) weight")
    B = f.shape[0]
    if out is None:
        out = torch.empty(B, dtype=torch.int64, device=f.device)

    def vec1(t, dtype, what):  # (B,) of dtype, any positive stride (a column of (B, 2) rows)
        if t.dtype != dtype or t.dim() != 1 or t.shape[0] != B or t.stride(0) < 1:
            raise ValueError(f"{what} must be ({B},) {dtype}")
        return t

    vec1(out, torch.int64, "out")
    if out16 is not None:
        vec1(out16, torch.int16, "out16")
    eps = torch.as_tensor(epsilon, dtype=torch.float32, device=f.device)
    tg = torch.as_tensor(tag, dtype=torch.int64, device=f.device)
    b = bias.contiguous()
    addcol, rows = None, None
    if move1 is not None:
        rows = move1 if move1.dtype == torch.int64 else move1.to(torch.int64)
        vec1(rows, torch.int64, "move1")
        addcol = weight.data_ptr() + 256 * weight.element_size()
    lib = _lib.load()
    _lib.check(lib.narde_head_policy576_dev(
        f.device.index, _lib.ptr(f), f.stride(0), 256, _lib.ptr(weight), weight.stride(0), _lib.ptr(b),
        _lib.ptr(mask576.contiguous()), B, _lib.ptr(eps), int(seed) & (2 ** 64 - 1), _lib.ptr(tg), int(head),
        addcol, _lib.ptr(rows), rows.stride(0) if rows is not None else 1, _lib.ptr(out), out.stride(0),
        _lib.ptr(out16), out16.stride(0) if out16 is not None else 1,
        ctypes.c_void_p(torch.cuda.current_stream(f.device).cuda_stream)), "narde_head_policy576_dev")
    return out


TUNED_GEMMS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tunableop_gfx950.csv")


def use_tuned_gemms(path=TUNED_GEMMS):
    """Select the driver's fp32 GEMMs (hipBLASLt / rocBLAS solutions per
    shape) from a TunableOp results file measured on MI355X (tools/diag/
    gpu_tunable.sh; torch validates the ROCm / hipBLASLt versions in it and
    falls back to its heuristics on a mismatch).  Process-wide torch state,
    so an application opt-in (bench.py), not a side effect of the driver.
    Returns whether the file was loaded."""
    if not os.path.exists(path):
        return False
    torch.cuda.tunable.enable(True)
    torch.cuda.tunable.tuning_enable(False)
    torch.cuda.tunable.set_filename(path, insert_device_ordinal=False)
    return bool(torch.cuda.tunable.read_file(path))


def _stream(dev):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _f32(x):
    if x.dtype != torch.float32 or not x.is_contiguous():
        raise ValueError("expected a contiguous float32 tensor")
    return _lib.ptr(x)


def rowmax_addend(base, tab, rows, out=None):
    """max_c base[i][c] + tab[rows[i]][c] over the 576 codes (k_rowmax_addend):
    the target move-2 head's max without the (B,576) sum."""
    n = base.shape[0]
    if base.stride(1) != 1 or tab.stride(1) != 1 or base.shape[1] != MOVES or tab.shape[1] != MOVES:
        raise ValueError("base / tab must be (., 576) float32 with unit column stride")
    rows = rows.to(torch.int64).contiguous()
    if out is None:
        out = torch.empty(n, dtype=torch.float32, device=base.device)
    _lib.check(_lib.load().narde_rowmax_addend(
        base.device.index, _lib.ptr(base), base.stride(0), _lib.ptr(tab), tab.stride(0), _lib.ptr(rows), n,
        _lib.ptr(out), _stream(base.device)), "narde_rowmax_addend")
    return out


def target_max2(nq1, base, tab, m1=None, am1=None, m2=None):
    """(m1, am1, m2): nq1.max(1) (values, indices: torch's rules -- NaN wins,
    ties to the lowest code) and rowmax_addend(base, tab, am1) in one launch
    (k_target_max2)."""
    n = nq1.shape[0]
    for t in (nq1, base, tab):
        if t.dtype != torch.float32 or t.stride(1) != 1 or t.shape[1] != MOVES:
            raise ValueError("nq1 / base / tab must be (., 576) float32 with unit column stride")
    z = dict(device=nq1.device)
    m1 = torch.empty(n, dtype=torch.float32, **z) if m1 is None else m1
    m2 = torch.empty(n, dtype=torch.float32, **z) if m2 is None else m2
    am1 = torch.empty(n, dtype=torch.int64, **z) if am1 is None else am1
    _lib.check(_lib.load().narde_target_max2(
        nq1.device.index, _lib.ptr(nq1), nq1.stride(0), _lib.ptr(base), base.stride(0), _lib.ptr(tab), tab.stride(0),
        n, _f32(m1), _lib.ptr(am1), _f32(m2), _stream(nq1.device)), "narde_target_max2")
    return m1, am1, m2


def learner_variant(flags):
    """narde_learner_variant: bit 1 = the float4 clip + Adam (default), else
    round 5's scalar passes; returns the previous flags."""
    return int(_lib.load().narde_learner_variant(int(flags)))


class GatheredHeads(torch.autograd.Function):
    """(q1, q2) = the online heads at the stored codes a (B,2):
    model.move1_head(f).gather(1, a[:, :1]) and
    model.move2_from_features(f, a[:, 0]).gather(1, a[:, 1:]), squeezed --
    the only entries the loss reads (train_deepq_pytorch.py:653-720).
    Forward and backward are three HIP kernels (narde_dqn_heads_forward /
    _backward: per-row dot products; per-code sums over the rows holding the
    code, deterministic) instead of the two dense (B,256)x(256,576) heads,
    their backward GEMMs, the bias-grad reductions and the gather/scatter
    and index_add chains autograd builds around them."""

    @staticmethod
    def forward(ctx, f, w1, b1, w2, b2, a):
        n = f.shape[0]
        if f.dtype != torch.float32 or f.dim() != 2 or f.shape[1] != 256 or f.stride(1) != 1:
            raise ValueError("f must be (B, 256) float32 with unit column stride")
        if tuple(w1.shape) != (MOVES, 256) or tuple(w2.shape) != (MOVES, 256 + MOVES):
            raise ValueError("w1 (576, 256), w2 (576, 832)")
        if not (w1.is_contiguous() and w2.is_contiguous() and b1.is_contiguous() and b2.is_contiguous()):
            raise ValueError("contiguous head parameters")
        a = a.contiguous()
        if a.dtype != torch.int64 or tuple(a.shape) != (n, 2):
            raise ValueError("a must be (B, 2) int64")
        q1 = torch.empty(n, dtype=torch.float32, device=f.device)
        q2 = torch.empty_like(q1)
        _lib.check(_lib.load().narde_dqn_heads_forward(
            f.device.index, _lib.ptr(f), f.stride(0), _lib.ptr(w1), w1.stride(0), _lib.ptr(b1), _lib.ptr(w2),
            w2.stride(0), _lib.ptr(b2), _lib.ptr(a), n, _lib.ptr(q1), _lib.ptr(q2), _stream(f.device)),
            "narde_dqn_heads_forward")
        ctx.save_for_backward(f, w1, w2, a)
        return q1, q2

    @staticmethod
    def backward(ctx, g1, g2):
        f, w1, w2, a = ctx.saved_tensors
        n = f.shape[0]
        # (torch materialises an unused output's grad as zeros; a broadcast
        # grad arrives with stride 0)
        g1, g2 = g1.to(torch.float32).contiguous(), g2.to(torch.float32).contiguous()
        gf = torch.empty((n, 256), dtype=torch.float32, device=f.device)
        gw1, gw2 = torch.empty_like(w1), torch.empty_like(w2)
        gb1 = torch.empty(MOVES, dtype=torch.float32, device=f.device)
        gb2 = torch.empty_like(gb1)
        _lib.check(_lib.load().narde_dqn_heads_backward(
            f.device.index, _lib.ptr(g1), _lib.ptr(g2), _lib.ptr(f), f.stride(0), _lib.ptr(w1), w1.stride(0), _lib.ptr(w2),
            w2.stride(0), _lib.ptr(a), n, _lib.ptr(gf), _lib.ptr(gw1), _lib.ptr(gb1), _lib.ptr(gw2),
            _lib.ptr(gb2), _stream(f.device)), "narde_dqn_heads_backward")
        return gf, gw1, gb1, gw2, gb2, None


def gathered_heads(model, f, a):
    """GatheredHeads.apply on a DecomposedDQN's heads."""
    h1, h2 = model.move1_head, model.move2_head
    return GatheredHeads.apply(f, h1.weight, h1.bias, h2.weight, h2.bias, a)


class LinearReLU(torch.autograd.Function):
    """relu(x W^T + b) (one of DecomposedDQN.feature_network's Linear + ReLU
    pairs) with the backward's ReLU mask and bias gradient in one HIP kernel
    (narde_relu_bias_grad: deterministic column sums) instead of autograd's
    threshold_backward + column reduction; the two GEMMs stay hipBLASLt.
    `scratch`: a device buffer for the kernel (relu_bias_grad_scratch)."""

    @staticmethod
    def forward(ctx, x, w, b, scratch):
        h = torch._addmm_activation(b, x, w.t())
        ctx.save_for_backward(x, w, h)
        ctx.scratch = scratch
        return h

    @staticmethod
    def backward(ctx, gh):
        x, w, h = ctx.saved_tensors
        gh = gh.contiguous()
        n, cols = h.shape
        g = torch.empty_like(h)
        db = torch.empty(cols, dtype=torch.float32, device=h.device)
        sc = ctx.scratch
        if sc.numel() < -(-n // 64) * cols:
            raise ValueError("relu_bias_grad scratch too small")
        _lib.check(_lib.load().narde_relu_bias_grad(
            h.device.index, _f32(gh), _f32(h), n, cols, _lib.ptr(g), _lib.ptr(db), _f32(sc), _stream(h.device)),
            "narde_relu_bias_grad")
        dx = g @ w if ctx.needs_input_grad[0] else None
        return dx, g.t() @ x, db, None


def relu_bias_grad_scratch(rows, cols, device):
    """The scratch narde_relu_bias_grad needs for (rows, cols)."""
    return torch.empty(-(-rows // 64) * cols, dtype=torch.float32, device=device)


def features_fused(model, x, scratch):
    """model.features(x) as two LinearReLU layers (same parameters, same
    forward values; gradients to fp32 rounding)."""
    l1, l2 = model.feature_network[0], model.feature_network[2]
    h = LinearReLU.apply(x, l1.weight, l1.bias, scratch)
    return LinearReLU.apply(h, l2.weight, l2.bias, scratch)


class DQNLoss(torch.autograd.Function):
    """The decomposed loss of train_deepq_pytorch.py:653-720 as one kernel
    (k_dqn_loss): forward returns the loss and writes the TD errors into
    `td`; the saved dloss/dq1, dloss/dq2 make the backward one multiply."""

    @staticmethod
    def compute(q1, q2, m1, m2, r, d, w, gamma, td, loss_copy):
        """(loss, dloss/dq1, dloss/dq2) without autograd: the learner hands
        the gradients to torch.autograd.backward((q1, q2), (g1, g2)) itself
        (the backward's `go * g` multiplies are two launches for go = 1)."""
        B = q1.shape[0]
        loss = torch.empty((), dtype=torch.float32, device=q1.device)
        g1, g2 = torch.empty_like(q1), torch.empty_like(q2)
        _lib.check(_lib.load().narde_dqn_loss(
            q1.device.index, _f32(q1), _f32(q2), _f32(m1), _f32(m2), _f32(r), _f32(d), _f32(w), B,
            float(gamma), _f32(td), _lib.ptr(loss), None if loss_copy is None else _f32(loss_copy),
            _lib.ptr(g1), _lib.ptr(g2), _stream(q1.device)), "narde_dqn_loss")
        return loss, g1, g2

    @staticmethod
    def forward(ctx, q1, q2, m1, m2, r, d, w, gamma, td, loss_copy):
        loss, g1, g2 = DQNLoss.compute(q1, q2, m1, m2, r, d, w, gamma, td, loss_copy)
        ctx.save_for_backward(g1, g2)
        return loss

    @staticmethod
    def backward(ctx, go):
        g1, g2 = ctx.saved_tensors
        return go * g1, go * g2, None, None, None, None, None, None, None, None


class FusedAdamClip:
    """clip_grad_norm_(max_norm) + torch.optim.Adam.step in two HIP kernels
    (narde_adam_clip): the gradient norm over all tensors with a
    deterministic last-block sum, then every element's clipped Adam update.
    Same math as torch's Adam (lerp first moment, bias corrections from a
    device step counter), fp32; graph-capturable (all state on device)."""

    def __init__(self, params, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, max_norm=10.0):
        self.params = [p for p in params]
        if not 1 <= len(self.params) <= 8:
            raise ValueError("1..8 parameter tensors")
        for p in self.params:
            if p.dtype != torch.float32 or not p.is_contiguous():
                raise ValueError("contiguous float32 parameters")
        self.lr, self.betas, self.eps, self.max_norm = float(lr), betas, float(eps), float(max_norm)
        self.m = [torch.zeros_like(p) for p in self.params]
        self.v = [torch.zeros_like(p) for p in self.params]
        dev = self.params[0].device
        self.step_t = torch.zeros((), dtype=torch.int64, device=dev)
        self.scratch = torch.zeros(1026, dtype=torch.float32, device=dev)
        n = len(self.params)
        self._sizes = (ctypes.c_int64 * n)(*[p.numel() for p in self.params])

    def zero_grad(self, set_to_none=True):
        for p in self.params:
            p.grad = None if set_to_none else (p.grad.zero_() if p.grad is not None else None)

    def step(self):
        n = len(self.params)
        grads = [p.grad for p in self.params]
        if any(g is None or not g.is_contiguous() or g.dtype != torch.float32 for g in grads):
            raise ValueError("every parameter needs a contiguous float32 .grad")
        arr = lambda ts: (ctypes.c_void_p * n)(*[t.data_ptr() for t in ts])  # noqa: E731
        dev = self.params[0].device
        _lib.check(_lib.load().narde_adam_clip(
            dev.index, n, arr(self.params), arr(grads), arr(self.m), arr(self.v), self._sizes,
            _lib.ptr(self.step_t), self.lr, float(self.betas[0]), float(self.betas[1]), self.eps, self.max_norm,
            _lib.ptr(self.scratch), _stream(dev)), "narde_adam_clip")


class DeviceReplay:
    """PrioritizedReplayBuffer (train_deepq_pytorch.py:279-342) on device
    tensors: new transitions get the running max priority, sampling is
    proportional to priority**alpha, importance weights (N p)^-beta / max,
    beta anneals by beta_increment per sample, priorities = |td| + epsilon.

    Layout (each observation stored once): the driver adds `stride` (= B,
    its env count) transitions per step, env i at row (pos + i) % capacity,
    so row j's next observation s' is the s of the same env's next
    transition, row (j + stride) % capacity.  A step writes its transitions'
    (a, r, done) and priority into rows whose s is already there (the
    previous step's s', or seed()), and its s' into the next `stride` rows,
    whose priority stays 0 -- never sampled -- until the next step completes
    them.  So `capacity - stride` transitions are live at most
    (capacity >= 2 * stride), `size` counts them, and sampling runs over the
    first `rows` rows.

    The write cursor, beta and the max priority live in device scalars and
    are updated in place, so add/sample/update can be captured in a graph
    (`pos` / `size` are host mirrors; sample() needs `rows` fixed, i.e. a
    full ring, to be replayed)."""

    def __init__(self, capacity, state_size, device, stride, alpha=0.6, beta=0.4, beta_increment=0.001,
                 epsilon=0.01):
        self.capacity, self.stride, self.device = int(capacity), int(stride), device
        if self.stride < 1 or self.capacity < 2 * self.stride:
            raise ValueError("capacity must be at least twice the transitions per step (stride)")
        self.alpha, self.beta_increment, self.epsilon = alpha, beta_increment, epsilon
        z = dict(device=device)
        self.obs = torch.zeros((self.capacity, state_size), dtype=torch.float32, **z)
        self.action = torch.zeros((self.capacity, 2), dtype=torch.int64, **z)
        self.reward = torch.zeros(self.capacity, dtype=torch.float32, **z)
        self.done = torch.zeros(self.capacity, dtype=torch.float32, **z)
        self.prio = torch.zeros(self.capacity, dtype=torch.float32, **z)  # 0: empty / pending rows
        self.max_prio = torch.ones((), dtype=torch.float32, **z)
        self.beta_t = torch.full((), beta, dtype=torch.float64, **z)
        self.pos_t = torch.zeros((), dtype=torch.int64, **z)
        self.sample_ctr = torch.zeros((), dtype=torch.int64, **z)  # k_per_sample's Philox counter
        self._sample_scratch = torch.zeros(2, dtype=torch.int32, **z)  # its grid max + ticket
        self._chunk = torch.empty((self.capacity + 1023) // 1024, dtype=torch.float32, **z)  # narde_per_prefix
        self.pos = 0
        self.size = 0

    @property
    def beta(self):
        return float(self.beta_t)

    @property
    def rows(self):
        """Rows sampling runs over: the live transitions plus the pending s' rows."""
        return min(self.size + self.stride, self.capacity) if self.size else 0

    def next_index(self, idx):
        """Row of each transition's next observation s'."""
        return (idx + self.stride) % self.capacity

    def seed(self, obs):
        """Write the observations s of the transitions the next step adds
        (rows pos .. pos + stride - 1, priority 0 until completed)."""
        idx = (torch.arange(self.stride, device=self.device) + self.pos_t) % self.capacity
        self.obs.index_copy_(0, idx, obs)
        self.prio.index_fill_(0, idx, 0.0)

    def add(self, action, reward, next_obs, done):
        """One step's `stride` transitions: k_dqn_transition's ring writes in
        torch ops (the restatement it is tested against)."""
        n = action.shape[0]
        if n != self.stride:
            raise ValueError("add() takes one step: stride transitions")
        idx = (torch.arange(n, device=self.device) + self.pos_t) % self.capacity
        self.action.index_copy_(0, idx, action)
        self.reward.index_copy_(0, idx, reward)
        self.done.index_copy_(0, idx, done)
        self.prio.index_copy_(0, idx, self.max_prio.expand(n))
        nidx = self.next_index(idx)
        self.obs.index_copy_(0, nidx, next_obs)
        self.prio.index_fill_(0, nidx, 0.0)
        self.pos_t.add_(n).remainder_(self.capacity)
        self.advance(n)

    def advance(self, n):
        """Host mirrors of one add() of n rows (also called per graph replay)."""
        self.pos = (self.pos + n) % self.capacity
        self.size = min(self.size + n, self.capacity - self.stride)

    def sample(self, batch, generator=None):
        n = self.rows
        p = self.prio[:n] ** self.alpha
        cdf = torch.cumsum(p, 0)
        total = cdf[-1]
        # inverse-CDF sampling (torch.multinomial over 1M categories spends
        # ~0.5 ms renormalising one huge row); pending rows have p = 0
        u = torch.rand(batch, device=p.device, generator=generator) * total
        idx = nearest_positive(p, torch.searchsorted(cdf, u, right=True).clamp_(max=n - 1))
        probs_idx = p[idx] / total
        w = (n * probs_idx) ** (-self.beta_t)
        w = w / w.max()
        self.beta_t.add_(self.beta_increment).clamp_(max=1.0)
        return idx, w

    def update(self, idx, td):
        pr = td + self.epsilon
        self.prio.index_copy_(0, idx, pr)
        torch.maximum(self.max_prio, pr.max(), out=self.max_prio)

    # ---- fused (HIP) learner path: the same rules, one kernel each
    def prefix(self, n):
        """(prio[:n] ** alpha, its inclusive prefix sum) in two launches
        (narde_per_prefix, round 6; sample() keeps torch's pow + cumsum,
        equal up to the rounding of the sums' association)."""
        p = torch.empty(n, dtype=torch.float32, device=self.prio.device)
        cdf = torch.empty_like(p)
        _lib.check(_lib.load().narde_per_prefix(
            p.device.index, _lib.ptr(self.prio), n, float(self.alpha), _lib.ptr(p), _lib.ptr(cdf),
            _lib.ptr(self._chunk), self._chunk.numel(), _stream(p.device)), "narde_per_prefix")
        return p, cdf

    def sample_fused(self, batch, seed, u_out=None):
        """sample() as k_per_sample: priority^alpha and its prefix sum
        (prefix()), then the search, weights and beta step in one kernel with
        its own device Philox counter (`sample_ctr`)."""
        n = self.rows
        p, cdf = self.prefix(n)
        idx = torch.empty(batch, dtype=torch.int64, device=p.device)
        w = torch.empty(batch, dtype=torch.float32, device=p.device)
        _lib.check(_lib.load().narde_per_sample(
            p.device.index, _lib.ptr(p), _lib.ptr(cdf), n, batch, int(seed) & (2 ** 64 - 1),
            _lib.ptr(self.sample_ctr), _lib.ptr(self.beta_t), float(self.beta_increment), _lib.ptr(idx),
            _lib.ptr(w), None if u_out is None else _f32(u_out), _lib.ptr(self._sample_scratch),
            _stream(p.device)), "narde_per_sample")
        return idx, w

    def sample_gather_fused(self, batch, seed):
        """sample_fused + gather in one launch (k_per_sample_gather): (idx, w,
        s, ns, a, r, d) with w UNNORMALISED -- loss_prio_fused normalises it
        in place and steps beta and the sampling counter."""
        n, ss = self.rows, self.obs.shape[1]
        p, cdf = self.prefix(n)
        z = dict(device=p.device)
        idx = torch.empty(batch, dtype=torch.int64, **z)
        w = torch.empty(batch, dtype=torch.float32, **z)
        s = torch.empty((batch, ss), dtype=torch.float32, **z)
        ns = torch.empty((batch, ss), dtype=torch.float32, **z)
        a = torch.empty((batch, 2), dtype=torch.int64, **z)
        r = torch.empty(batch, dtype=torch.float32, **z)
        d = torch.empty(batch, dtype=torch.float32, **z)
        _lib.check(_lib.load().narde_per_sample_gather(
            p.device.index, _lib.ptr(p), _lib.ptr(cdf), n, batch, int(seed) & (2 ** 64 - 1), _lib.ptr(self.sample_ctr),
            _lib.ptr(self.beta_t), _lib.ptr(idx), _lib.ptr(w), ss, _lib.ptr(self.obs), self.stride, self.capacity,
            _lib.ptr(self.action), _lib.ptr(self.reward), _lib.ptr(self.done), _lib.ptr(s), _lib.ptr(ns), _lib.ptr(a),
            _lib.ptr(r), _lib.ptr(d), _stream(p.device)), "narde_per_sample_gather")
        return idx, w, s, ns, a, r, d

    def loss_prio_fused(self, q1, q2, m1, m2, r, d, w, gamma, td, loss, idx, epsilon=None, eps_min=0.0,
                        eps_decay=1.0, cursor_add=0, tag=None):
        """DQNLoss.compute + update_fused + sample_fused's normalisation and
        beta / counter steps in one block (k_dqn_loss_prio); w (raw, from
        sample_gather_fused) is normalised in place.  Returns (g1, g2)."""
        B = q1.shape[0]
        g1, g2 = torch.empty_like(q1), torch.empty_like(q2)
        _lib.check(_lib.load().narde_dqn_loss_prio(
            q1.device.index, _f32(q1), _f32(q2), _f32(m1), _f32(m2), _f32(r), _f32(d), _f32(w), B, float(gamma),
            _f32(td), _lib.ptr(loss), None, _lib.ptr(g1), _lib.ptr(g2), _lib.ptr(idx), float(self.epsilon),
            _lib.ptr(self.prio), _lib.ptr(self.max_prio), None if epsilon is None else _lib.ptr(epsilon),
            float(eps_min), float(eps_decay), _lib.ptr(self.pos_t) if cursor_add else None, int(cursor_add),
            self.capacity, _lib.ptr(tag), _lib.ptr(self.sample_ctr), _lib.ptr(self.beta_t), float(self.beta_increment),
            _stream(q1.device)), "narde_dqn_loss_prio")
        return g1, g2

    def gather(self, idx):
        """(s, ns, a, r, d) rows of idx (k_gather_batch; ns from row
        next_index(idx))."""
        B, ss = idx.shape[0], self.obs.shape[1]
        z = dict(device=self.obs.device)
        s = torch.empty((B, ss), dtype=torch.float32, **z)
        ns = torch.empty((B, ss), dtype=torch.float32, **z)
        a = torch.empty((B, 2), dtype=torch.int64, **z)
        r = torch.empty(B, dtype=torch.float32, **z)
        d = torch.empty(B, dtype=torch.float32, **z)
        _lib.check(_lib.load().narde_gather_batch(
            self.obs.device.index, _lib.ptr(idx), B, ss, _lib.ptr(self.obs), self.stride, self.capacity,
            _lib.ptr(self.action), _lib.ptr(self.reward), _lib.ptr(self.done), _lib.ptr(s), _lib.ptr(ns),
            _lib.ptr(a), _lib.ptr(r), _lib.ptr(d), _stream(self.obs.device)), "narde_gather_batch")
        return s, ns, a, r, d

    def update_fused(self, idx, td, epsilon=None, eps_min=0.0, eps_decay=1.0, cursor_add=0, tag=None):
        """update() as k_prio_update (+ the driver's epsilon decay when an
        epsilon device scalar is given; + the write cursor's advance by
        cursor_add rows and the driver's step tag + 1, when given -- the
        step's bookkeeping folded into this launch)."""
        _lib.check(_lib.load().narde_prio_update(
            idx.device.index, _lib.ptr(idx), _f32(td), idx.shape[0], float(self.epsilon), _lib.ptr(self.prio),
            _lib.ptr(self.max_prio), None if epsilon is None else _lib.ptr(epsilon), float(eps_min),
            float(eps_decay), _lib.ptr(self.pos_t) if cursor_add else None, int(cursor_add), self.capacity,
            _lib.ptr(tag), _stream(idx.device)), "narde_prio_update")


class BatchedDQNDriver:
    """B envs of DQN self-play on one GPU; one call of step() = one env step
    for every env + `updates_per_step` prioritized DQN updates.

    All driver state (epsilon, the step tag, the replay cursor, beta, the
    max priority, the current observation) lives in device tensors updated
    in place, so a whole step -- masks, both policy heads, env step,
    shaping, replay write, minibatch sample, loss, backward, clip, Adam --
    can be captured once in a torch.cuda.CUDAGraph and replayed
    (capture_graph()); the replay then costs one launch instead of ~150.
    The target-network sync stays on the host (every target_update
    updates, an in-place copy the graph reads)."""

    def __init__(self, env, obs="tesauro198", train_batch=4096, capacity=1 << 20,
                 learning_rate=1e-4, gamma=0.99, epsilon=1.0, epsilon_min=0.01,
                 epsilon_decay=0.995, target_update=10, updates_per_step=1, shaping=True,
                 seed=0, fused=True, fused_heads=True, gathered_heads=True, fused_features=True,
                 explore="plays", greedy="accepted", one_launch_chains=True):
        if env.full:
            raise ValueError("the DQN driver plays the reference's (move1, move2) actions: rules='ref2'")
        if explore not in ("plays", "codes"):
            raise ValueError("explore must be 'plays' (the reference's act()) or 'codes'")
        # the epsilon-branch law: "plays" = random.choice over act()'s
        # (move1, move2) combinations (train_deepq_pytorch.py:430-515, second
        # moves listed on the pre-move board), k_explore_plays; "codes" = each
        # head uniform over its own legal codes (the policy kernels alone)
        self.explore = explore
        if greedy not in ("accepted", "reference"):
            raise ValueError("greedy must be 'accepted' or 'reference'")
        # the greedy branch's candidate sets: "accepted" = the codes the step
        # executes (move 1 it accepts, move 2 it accepts after that move 1,
        # post-move); "reference" = act()'s own (valid_first_moves' keys,
        # then valid_first_moves[move1]: pre-move lists, :520-560)
        self.greedy = greedy
        self.env, self.dev = env, env.device
        self.obs_kind = obs
        self.state_size = 198 if obs == "tesauro198" else 24
        torch.manual_seed(seed)
        self.gen = torch.Generator(device=self.dev)
        self.gen.manual_seed(seed)
        self.model = DecomposedDQN(self.state_size).to(self.dev)
        self.target = DecomposedDQN(self.state_size).to(self.dev)
        self.target.load_state_dict(self.model.state_dict())
        # capturable: the step count and bias corrections stay on the device
        self.opt = torch.optim.Adam(self.model.parameters(), lr=learning_rate, capturable=True, fused=True)
        # the fused learner's clip + Adam (two kernels instead of ~12 launches)
        self.fopt = FusedAdamClip(self.model.parameters(), lr=learning_rate, max_norm=10.0) if fused else None
        self.replay = DeviceReplay(capacity, self.state_size, self.dev, stride=env.num_envs)
        self.train_batch, self.gamma = int(train_batch), gamma
        z = dict(device=self.dev)
        self.eps_t = torch.full((), epsilon, dtype=torch.float32, **z)
        self.epsilon_min, self.epsilon_decay = epsilon_min, epsilon_decay
        self.target_update, self.updates_per_step = target_update, updates_per_step
        self.shaping = shaping
        # k_dqn_transition: observation + shaping + replay write in one kernel
        # (the 198-float observation only; the torch restatement otherwise)
        self.fused = bool(fused) and obs == "tesauro198"
        self.fused_learner = bool(fused)
        # the policy heads computed in the policy kernel (legal codes only)
        self.fused_heads = bool(fused_heads)
        # the fused learner's online heads at the stored codes only
        # (GatheredHeads) instead of dense heads + gather
        self.gathered_heads = bool(gathered_heads)
        # ... and its feature layers' ReLU mask + bias gradients in one kernel
        # each (LinearReLU)
        self.fused_features = bool(fused_features)
        # round 6: the learner's one-block / one-launch chains (_update_fused6)
        self.one_launch_chains = bool(one_launch_chains)
        self._rb_scratch = relu_bias_grad_scratch(self.train_batch, 256, self.dev)
        self.seed = seed
        self.tag_t = torch.zeros((), dtype=torch.int64, **z)
        self.steps = 0
        self.train_steps = 0
        B = env.num_envs
        self.off_seen = torch.zeros((B, 2), dtype=torch.float32, **z)
        self.state = self._observe()
        self._next = torch.empty_like(self.state)
        self.misc = self._misc_now()
        self.replay.seed(self.state)
        self.loss_t = torch.zeros((), dtype=torch.float32, **z)
        self.last_loss = None
        self.graph = None
        self._capturing = False
        self._fold = None  # (cursor rows, tag) the next fused update advances
        self._wm_rows, self._wm_ver = None, -1  # _target_onehot_rows' cache

    @property
    def epsilon(self):
        return float(self.eps_t)

    # ---------------------------------------------------------------- env side
    def _observe(self, out=None):
        if self.obs_kind == "tesauro198":
            if out is None:
                return self.env.tesauro198().clone()
            return self.env.tesauro198(out=out)
        x = self.env.observe().to(torch.float32)
        return x if out is None else out.copy_(x)

    def _misc_now(self):
        """(B,) int32 off_white | off_black << 4 | black_to_move << 10 of
        every env's record now (k_dqn_transition's misc word)."""
        st = self.env.get_state()
        off = st["off"].to(torch.int32)
        return off[:, 0] | (off[:, 1] << 4) | ((st["player"] == -1).to(torch.int32) << 10)

    def resync(self):
        """After the env was stepped or reset outside the driver: observe
        the current state again and make it the s of the next transitions."""
        self.state.copy_(self._observe())
        self.misc.copy_(self._misc_now())
        self.replay.seed(self.state)

    @torch.no_grad()
    def act(self, x):
        """Masked epsilon-greedy (move1, move2) codes for the next step: the
        env's exact legal masks and the fused policy kernel (epsilon and the
        step tag read from device memory).  Greedy (greedy="accepted"):
        move 1 = the masked argmax over the move-1 codes the step accepts,
        move 2 = the masked argmax over the codes the step accepts after it
        (post-move); greedy="reference": over act()'s own candidate sets
        (narde_act_masks: list #1's codes, then the pre-move second list of
        that move 1, :520-560).
        Ties (parity unpinned): the policy kernels break an exact Q tie by
        the LOWEST code; act()'s torch.argmax over valid_first_moves' keys
        breaks it by insertion order (list #1: the higher die's sources
        first, then the lower die's, :527-539), so on tied or NaN Q-values
        move 1 may differ from the reference.  The 2,500-decision golden
        (act_greedy.npz, random fixed Q) has no ties.
        Exploring rows (one shared draw per row and step): explore="plays"
        draws one of act()'s (move1, move2) combinations uniformly
        (k_explore_plays), as random.choice(valid_move_combinations)."""
        f = self.model.features_nograd(x)
        if self.fused_heads:
            # both heads inside the policy kernel, legal codes only
            # (k_head_policy576): no dense (B,256)x(256,576) GEMM per head
            # codes written straight into the (B, 2) action rows (and move 1
            # as int16 for the move-2 mask): no stack / dtype-cast kernels
            h1, h2 = self.model.move1_head, self.model.move2_head
            acts = torch.empty((x.shape[0], 2), dtype=torch.int64, device=self.dev)
            m1 = torch.empty(x.shape[0], dtype=torch.int16, device=self.dev)
            ref = self.greedy == "reference"
            head_policy_576(f, h1.weight, h1.bias, self.env.act_masks() if ref else self.env.legal_mask(),
                            self.eps_t, self.seed, self.tag_t, 0, out=acts[:, 0], out16=m1)
            m2 = self.env.act_masks(move1=acts[:, 0]) if ref else self.env.legal_mask_move2(m1)
            head_policy_576(f, h2.weight, h2.bias, m2, self.eps_t, self.seed, self.tag_t, 1, out=acts[:, 1],
                            move1=acts[:, 0])
            if self.explore == "plays":
                self.env.explore_plays(acts, self.eps_t, self.seed, self.tag_t)
            return acts
        ref = self.greedy == "reference"
        a1 = policy_576(self.model.move1_head(f), self.env.act_masks() if ref else self.env.legal_mask(), self.eps_t,
                        self.seed, self.tag_t, 0)
        m2 = self.env.act_masks(move1=a1) if ref else self.env.legal_mask_move2(a1.to(torch.int16))
        # move-2 Q = (f @ Wf^T + b) + Wm[:, move1]: the column add is fused
        # into the policy kernel (rows of Wm^T, a 1.3 MB transpose per step)
        w = self.model.move2_head.weight
        base = torch.nn.functional.linear(f, w[:, :256], self.model.move2_head.bias)
        wm_rows = w[:, 256:].t().contiguous()
        a2 = policy_576(base, m2, self.eps_t, self.seed, self.tag_t, 1, add=(wm_rows, a1))
        acts = torch.stack([a1, a2], 1)
        if self.explore == "plays":
            self.env.explore_plays(acts, self.eps_t, self.seed, self.tag_t)
        return acts

    def step(self):
        """One env step for every env + the updates; returns the last loss
        (a device scalar) or None while the replay holds < train_batch."""
        if self.graph is not None:
            return self._replay_graph()
        loss = self._step_body()
        self._host_after_step(loss is not None)
        return self.last_loss if loss is not None else None

    def _step_body(self):
        """Everything one step runs on the device, host-sync free (the body
        capture_graph() records).  Host-side counters: _host_after_step."""
        x = self.state
        actions = self.act(x)
        _, reward, term, trunc, info = self.env.step(actions.to(torch.int16))
        # when the fused learner runs this step, the ring cursor's advance and
        # the step tag's increment ride in its last kernel (k_prio_update)
        n, rp = self.env.num_envs, self.replay
        if self.fused:
            self._transition_fused(actions, reward, term, trunc, info["legal"], advance_cursor=False)
        else:
            self._transition_torch(actions, reward, term, trunc, info["legal"])
        fold = self.fused_learner and self.updates_per_step >= 1 and rp.size >= self.train_batch
        if fold:
            self._fold = (n if self.fused else 0, self.tag_t)
        else:
            if self.fused:
                rp.pos_t.add_(n).remainder_(rp.capacity)
            self.tag_t.add_(1)
        loss = None
        for _ in range(self.updates_per_step):
            loss = self._update_body()
        return loss

    def _transition_torch(self, actions, reward, term, trunc, legal):
        """Shaping + replay write + s <- s' in torch ops (the restatement
        k_dqn_transition is tested against; the int24 observation path)."""
        r = reward.to(torch.float32)
        t, u = term.bool(), trunc.bool()
        done = (t | u).to(torch.float32)
        nxt = self._observe(out=self._next)
        post = self._misc_now()
        if self.shaping:
            # train_deepq_pytorch.py:892-912: +1 per checker newly borne off
            # and +0.1 x the count, for env.unwrapped.current_player read
            # AFTER the step -- at a step that ends the game (auto-reset has
            # already started the next one) the pre-step record's: the mover
            # (the winner, 15 off) if it terminated, the other player if
            # truncated; none without a legal move (:869-873)
            pre = self.misc
            moved = (legal & 0xFFFFFFFFFFFF) != 0
            pre_black = (pre >> 10) & 1
            black = torch.where(t, pre_black, torch.where(u, 1 - pre_black, (post >> 10) & 1)).long()
            src = torch.where(t | u, pre, post)
            cnt = torch.where(black == 1, (src >> 4) & 15, src & 15).to(torch.float32)
            now = torch.where(t, torch.full_like(cnt, 15.0), cnt)
            before = self.off_seen.gather(1, black.unsqueeze(1)).squeeze(1)
            r = torch.where(moved, r + (now - before).clamp(min=0) + 0.1 * now, r)
            seen = self.off_seen.scatter(1, black.unsqueeze(1), now.unsqueeze(1))
            self.off_seen.copy_(torch.where(moved.unsqueeze(1), seen, self.off_seen))
            self.off_seen.mul_((1.0 - done).unsqueeze(1))  # new episode: trackers restart at 0
        self.misc.copy_(post)
        self.replay.add(actions, r, nxt, done)
        self.state.copy_(nxt)

    def _transition_fused(self, actions, reward, term, trunc, legal, advance_cursor=True):
        rp, n = self.replay, self.env.num_envs
        if not (self.state.is_contiguous() and actions.is_contiguous() and actions.dtype == torch.int64):
            raise ValueError("state / actions layout")
        self.env.handle.call(
            "narde_dqn_transition", _lib.ptr(self.state), _lib.ptr(actions), _lib.ptr(reward),
            _lib.ptr(term), _lib.ptr(trunc), _lib.ptr(legal), _lib.ptr(self.misc), _lib.ptr(self.off_seen),
            int(self.shaping), _lib.ptr(rp.obs), _lib.ptr(rp.action), _lib.ptr(rp.reward), _lib.ptr(rp.done),
            _lib.ptr(rp.prio), _lib.ptr(rp.max_prio), _lib.ptr(rp.pos_t), rp.capacity,
            ctypes.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream))
        if advance_cursor:
            rp.pos_t.add_(n).remainder_(rp.capacity)
        rp.advance(n)

    def _host_after_step(self, trained):
        self.steps += 1
        if trained:
            self.last_loss = self.loss_t.clone()

    def capture_graph(self, warmup=3):
        """Record one step into a CUDA graph; later step() calls replay it.
        Needs a full replay ring after the warmup steps (sample() sizes are
        fixed in the graph) and one update per step (the host-side target
        sync runs between replays).  The warmup steps are real steps, run
        eagerly on a side stream as torch's capture rules ask."""
        if self.updates_per_step != 1:
            raise ValueError("graph capture needs updates_per_step == 1")
        cap, B = self.replay.capacity, self.env.num_envs
        # steps until the ring is full (size = capacity - B live transitions)
        need = max(0, -(-(cap - B - self.replay.size - warmup * B) // B))
        side = torch.cuda.Stream(self.dev)
        side.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(side):
            for _ in range(need + warmup):
                self.step()
        torch.cuda.current_stream(self.dev).wait_stream(side)
        if self.replay.rows != cap or self.replay.size < self.train_batch:
            raise RuntimeError("replay ring not full before capture")
        g = torch.cuda.CUDAGraph()
        g.register_generator_state(self.gen)
        # the captured body must not advance the host mirrors: replays do
        pos, size = self.replay.pos, self.replay.size
        self._capturing = True
        try:
            with torch.cuda.graph(g):
                self._step_body()
        finally:
            self._capturing = False
        self.replay.pos, self.replay.size = pos, size
        self.graph = g
        return self._replay_graph()  # capture does not execute: run it once

    def _replay_graph(self):
        self.graph.replay()
        self.replay.advance(self.env.num_envs)
        self._after_update()
        self._host_after_step(True)
        return self.last_loss

    # ------------------------------------------------------------ learner side
    def update(self):
        """DQNAgent.replay (train_deepq_pytorch.py:602-750), decomposed branch."""
        if self._update_body() is None:
            return None
        self.last_loss = self.loss_t.clone()
        return self.last_loss

    def _update_body(self):
        if self.replay.size < self.train_batch:
            return None
        if self.fused_learner:
            return self._update_fused()
        return self._update_torch()

    def _update_fused(self):
        """_update_torch with the non-GEMM chains as HIP kernels
        (csrc/dqn_learner.hip): sample, gather, target move-2 max, loss +
        grads, priorities + epsilon.  ~40 fewer launches per update.
        one_launch_chains (round 6, default): sample + gather in one launch,
        the target heads' max / argmax / move-2 max in one, and the weight
        normalisation + loss + priorities + bookkeeping in one block."""
        if self.one_launch_chains:
            return self._update_fused6()
        rp = self.replay
        idx, w = rp.sample_fused(self.train_batch, self.seed)
        s, ns, a, r, d = rp.gather(idx)
        f = features_fused(self.model, s, self._rb_scratch) if self.fused_features else self.model.features(s)
        if self.gathered_heads:
            q1, q2 = gathered_heads(self.model, f, a)
        else:
            q1 = self.model.move1_head(f).gather(1, a[:, :1]).squeeze(1)
            q2 = self.model.move2_from_features(f, a[:, 0]).gather(1, a[:, 1:]).squeeze(1)
        with torch.no_grad():
            tf = self.target.features_nograd(ns)
            m1, am1 = self.target.move1_head(tf).max(1)
            wt = self.target.move2_head.weight
            base2 = torch.nn.functional.linear(tf, wt[:, :256], self.target.move2_head.bias)
            m2 = rowmax_addend(base2, self._target_onehot_rows(), am1)
        td = torch.empty_like(r)
        _, g1, g2 = DQNLoss.compute(q1.detach(), q2.detach(), m1, m2, r, d, w, self.gamma, td, self.loss_t)
        self.fopt.zero_grad(set_to_none=True)
        torch.autograd.backward((q1, q2), (g1, g2))  # = loss.backward(): dloss/dq from k_dqn_loss
        self.fopt.step()  # clip_grad_norm_(10) + Adam
        cursor_add, tag = self._fold if self._fold is not None else (0, None)
        self._fold = None
        rp.update_fused(idx, td, self.eps_t, self.epsilon_min, self.epsilon_decay, cursor_add=cursor_add, tag=tag)
        if self._capturing:
            return self.loss_t
        self._after_update()
        return self.loss_t

    def _update_fused6(self):
        rp = self.replay
        idx, w, s, ns, a, r, d = rp.sample_gather_fused(self.train_batch, self.seed)
        f = features_fused(self.model, s, self._rb_scratch) if self.fused_features else self.model.features(s)
        if self.gathered_heads:
            q1, q2 = gathered_heads(self.model, f, a)
        else:
            q1 = self.model.move1_head(f).gather(1, a[:, :1]).squeeze(1)
            q2 = self.model.move2_from_features(f, a[:, 0]).gather(1, a[:, 1:]).squeeze(1)
        with torch.no_grad():
            tf = self.target.features_nograd(ns)
            nq1 = self.target.move1_head(tf)
            wt = self.target.move2_head.weight
            # (one GEMM of both heads' 1,152 columns measured slower: hipBLASLt
            # picks a 64x32 tile for it, 41.8 against 17.8 + 19.6 us)
            base2 = torch.nn.functional.linear(tf, wt[:, :256], self.target.move2_head.bias)
            m1, _, m2 = target_max2(nq1, base2, self._target_onehot_rows())
        td = torch.empty_like(r)
        cursor_add, tag = self._fold if self._fold is not None else (0, None)
        self._fold = None
        g1, g2 = rp.loss_prio_fused(q1.detach(), q2.detach(), m1, m2, r, d, w, self.gamma, td, self.loss_t, idx,
                                    self.eps_t, self.epsilon_min, self.epsilon_decay, cursor_add=cursor_add, tag=tag)
        self.fopt.zero_grad(set_to_none=True)
        torch.autograd.backward((q1, q2), (g1, g2))  # = loss.backward(): dloss/dq from k_dqn_loss_prio
        self.fopt.step()  # clip_grad_norm_(10) + Adam
        if self._capturing:
            return self.loss_t
        self._after_update()
        return self.loss_t

    def _update_torch(self):
        """DQNAgent.replay (train_deepq_pytorch.py:602-750), decomposed
        branch, in torch ops (the restatement the fused path is tested
        against)."""
        idx, w = self.replay.sample(self.train_batch, generator=self.gen)
        s, ns = self.replay.obs[idx], self.replay.obs[self.replay.next_index(idx)]
        a, r, d = self.replay.action[idx], self.replay.reward[idx], self.replay.done[idx]
        f = self.model.features(s)
        q1 = self.model.move1_head(f).gather(1, a[:, :1]).squeeze(1)
        q2 = self.model.move2_from_features(f, a[:, 0]).gather(1, a[:, 1:]).squeeze(1)
        with torch.no_grad():
            tf = self.target.features(ns)
            nq1 = self.target.move1_head(tf)
            t1 = r + (1 - d) * self.gamma * nq1.max(1)[0]
            nq2 = self.target.move2_from_features(tf, nq1.argmax(1))
            t2 = r + (1 - d) * self.gamma * nq2.max(1)[0]
        td = torch.clamp((t1 - q1).abs() + (t2 - q2).abs(), 0.0, 100.0).detach()
        loss = (w * (q1 - t1) ** 2).mean() + (w * (q2 - t2) ** 2).mean()
        self.opt.zero_grad(set_to_none=True)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(self.model.parameters(), max_norm=10.0)
        self.opt.step()
        self.replay.update(idx, td)
        # epsilon decay per update (:745-746): if eps > eps_min: eps *= decay
        self.eps_t.copy_(torch.where(self.eps_t > self.epsilon_min, self.eps_t * self.epsilon_decay,
                                     self.eps_t))
        self.loss_t.copy_(loss.detach())
        if self._capturing:
            return self.loss_t  # the host-side bookkeeping below runs per replay
        self._after_update()
        return self.loss_t

    def _target_onehot_rows(self):
        """The target move-2 head's one-hot columns as rows (576, 576),
        cached: the target changes only at its sync (refreshed in place
        there, outside any captured graph), so the step does not copy 1.3 MB
        per update; a stale cache (weights changed in place elsewhere) is
        caught by the tensor's version counter."""
        wt = self.target.move2_head.weight
        if self._wm_rows is None or self._wm_ver != wt._version:
            self._wm_rows = wt[:, 256:].t().contiguous()
            self._wm_ver = wt._version
        return self._wm_rows

    def _after_update(self):
        self.train_steps += 1
        if self.train_steps % self.target_update == 0:
            self.target.load_state_dict(self.model.state_dict())
            if self._wm_rows is not None:  # in place: a captured graph holds its address
                wt = self.target.move2_head.weight
                self._wm_rows.copy_(wt[:, 256:].t())
                self._wm_ver = wt._version
