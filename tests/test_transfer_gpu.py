"""csrc/kernels/transfer.hip box copies against the same plans run through strided torch views:
packs of random sub-regions of 2-5 D tensors (contiguous and permuted sources) into one flat
buffer, the unpack back, and the add mode of partial-sum receives (fp32 / bf16); vector widths
from 16 B down to one element."""
import numpy as np
import pytest
import torch

from flexflow_amd.parallel import boxcopy

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _regions(rng, shape, n):
    out = []
    for _ in range(n):
        r = []
        for s in shape:
            lo = int(rng.integers(0, s))
            hi = int(rng.integers(lo + 1, s + 1))
            r.append((lo, hi))
        out.append(r)
    return out


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape,perm", [((64, 96), None), ((8, 12, 40), None), ((4, 6, 10, 24), (0, 2, 3, 1)),
                                        ((3, 5, 4, 6, 16), None), ((256, 1024), None)])
def test_pack_unpack_matches_views(dtype, shape, perm):
    rng = np.random.default_rng(len(shape) * 7 + (perm is not None))
    x = torch.randn(shape, device=DEV).to(dtype)
    if perm is not None:  # a non-contiguous source (channels-last style)
        x = torch.randn([shape[i] for i in np.argsort(perm)], device=DEV).to(dtype).permute(*perm)
        assert tuple(x.shape) == shape and not x.is_contiguous()
    regs = _regions(rng, shape, 7)
    if len(shape) == 2 and shape[1] == 1024:
        regs = [[(0, 256), (0, 512)], [(0, 128), (512, 1024)]]  # whole 16-B rows: the vector path
    boxes, off = [], 0
    for r in regs:
        so, ss, ext = boxcopy.region_box(x, r)
        boxes.append((so, ss) + boxcopy.flat_box(off, ext))
        off += int(np.prod(ext))
    flat = torch.full((off,), 7.0, device=DEV, dtype=dtype)
    plan = boxcopy.BoxPlan(boxes, x, flat)
    plan.run(x, flat)
    ref = torch.cat([x[tuple(slice(lo, hi) for lo, hi in r)].reshape(-1) for r in regs])
    assert torch.equal(flat, ref)
    if len(shape) == 2 and shape[1] == 1024:
        assert plan.vec * flat.element_size() == 16
    # the overlaps of a re-layout tile the destination: split every dim in halves, pack x's tiles,
    # unpack them into a fresh tensor of x's geometry — the round trip is the identity
    import itertools
    tiles = [list(t) for t in itertools.product(*[[(0, n // 2), (n // 2, n)] if n > 1 else [(0, n)] for n in shape])]
    boxes, off = [], 0
    for r in tiles:
        so, ss, ext = boxcopy.region_box(x, r)
        boxes.append((so, ss) + boxcopy.flat_box(off, ext))
        off += int(np.prod(ext))
    flat = torch.empty(off, device=DEV, dtype=dtype)
    boxcopy.BoxPlan(boxes, x, flat).run(x, flat)
    y = torch.full_like(x, 3.0)
    ub = [boxcopy.flat_box(b[2], b[4])[:2] + boxcopy.region_box(y, r) for b, r in zip(boxes, tiles)]
    boxcopy.BoxPlan(ub, flat, y).run(flat, y)
    assert torch.equal(y, x)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_add_mode_sums_partials(dtype):
    x = torch.randn(6, 10, 32, device=DEV).to(dtype)
    parts = [torch.randn(2, 10, 16, device=DEV).to(dtype) for _ in range(3)]
    flat = torch.cat([p.reshape(-1) for p in parts])
    regs = [[(0, 2), (0, 10), (0, 16)], [(2, 4), (0, 10), (16, 32)], [(4, 6), (0, 10), (8, 24)]]
    boxes, off = [], 0
    for r, p in zip(regs, parts):
        boxes.append(boxcopy.flat_box(off, p.shape)[:2] + boxcopy.region_box(x, r))
        off += p.numel()
    ref = x.clone()
    for r, p in zip(regs, parts):
        ref[tuple(slice(lo, hi) for lo, hi in r)] += p
    boxcopy.BoxPlan(boxes, flat, x).run(flat, x, add=True)
    tol = 0 if dtype == torch.float32 else 1e-2
    assert torch.allclose(x.float(), ref.float(), atol=tol, rtol=tol)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_add_mode_overlapping_boxes_do_not_race(dtype):
    """Partial-sum replicas all add into ONE region and 2-D halo gradients overlap at the corners:
    the plan splits such boxes into launches with disjoint destinations (one launch
    read-modify-wrote the same elements from different workgroups and lost updates)."""
    torch.manual_seed(4)
    x = torch.randn(64, 256, device=DEV).to(dtype)
    parts = [torch.randn(48, 192, device=DEV).to(dtype) for _ in range(6)]
    flat = torch.cat([p.reshape(-1) for p in parts])
    regs = [[(0, 48), (0, 192)]] * 4 + [[(16, 64), (64, 256)], [(8, 56), (32, 224)]]
    boxes, off = [], 0
    for r, p in zip(regs, parts):
        boxes.append(boxcopy.flat_box(off, p.shape)[:2] + boxcopy.region_box(x, r))
        off += p.numel()
    ref = x.float().clone()
    for r, p in zip(regs, parts):
        ref[tuple(slice(lo, hi) for lo, hi in r)] += p.float()
    plan = boxcopy.BoxPlan(boxes, flat, x)
    assert len(plan.add_layers) >= 4
    for _ in range(3):  # a race would lose a random subset of adds: compare every run
        y = x.clone()
        plan.run(flat, y, add=True)
        tol = 1e-5 if dtype == torch.float32 else 3e-2
        assert torch.allclose(y.float(), ref, atol=tol, rtol=tol)


def test_out_of_range_box_is_refused_on_the_host():
    x = torch.zeros(4, 8, device=DEV)
    flat = torch.zeros(16, device=DEV)
    with pytest.raises(ValueError):
        boxcopy.BoxPlan([(0, (8, 1), 0, (8, 1), (3, 8))], x, flat)  # 24 elements into 16


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cl", [False, True])
def test_concat_split_reverse_match_torch(dtype, cl):
    """Concat (one launch over up to 16 inputs, more in groups), dense Split and Reverse on the
    box kernel against torch.cat / torch.split / torch.flip."""
    torch.manual_seed(2)
    fmt = torch.channels_last if cl else torch.contiguous_format
    xs = [torch.randn(4, c, 5, 6, device=DEV).to(dtype).contiguous(memory_format=fmt) for c in (8, 16, 24, 8)]
    cache = {}
    out = boxcopy.concat(cache, xs, 1)
    assert torch.equal(out, torch.cat(xs, 1))
    assert out.is_contiguous(memory_format=fmt)
    many = [torch.randn(3, 8, device=DEV).to(dtype) for _ in range(37)]
    assert torch.equal(boxcopy.concat(cache, many, 1), torch.cat(many, 1))
    # rows of 5 elements do not vectorize: the caller keeps torch.cat
    assert boxcopy.concat(cache, [torch.randn(3, 5, device=DEV).to(dtype)] * 2, 1) is None
    parts = boxcopy.split_dense(cache, out, [8, 16, 24, 8], 1)
    for p, r in zip(parts, xs):
        assert torch.equal(p, r)
    for ax in range(4):
        assert torch.equal(boxcopy.reverse(cache, out, ax), torch.flip(out, [ax]))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("itype", [torch.int32, torch.int64])
@pytest.mark.parametrize("dim", [0, 1, 2])
def test_gather_kernels_match_torch(ffC, dtype, itype, dim):
    """transfer.hip gather forward and its scatter-add backward against torch.gather / scatter_add_
    (fp32 reference), repeated indices included."""
    torch.manual_seed(3)
    shp = [6, 7, 9]
    x = torch.randn(shp, device=DEV).to(dtype)
    ishp = list(shp)
    ishp[dim] = 5
    idx = torch.randint(0, shp[dim], ishp, device=DEV, dtype=itype)
    inner = 1
    for e in shp[dim + 1:]:
        inner *= e
    out = torch.empty(ishp, device=DEV, dtype=dtype)
    ffC.gather_fwd(x, idx, out, ishp[dim], inner, shp[dim])
    assert torch.equal(out, torch.gather(x, dim, idx.long()))
    dy = torch.randn(ishp, device=DEV).to(dtype)
    dx = torch.zeros(shp, device=DEV)
    ffC.gather_bwd(dy, idx, dx, ishp[dim], inner, shp[dim])
    ref = torch.zeros(shp, device=DEV).scatter_add_(dim, idx.long(), dy.float())
    assert torch.allclose(dx, ref, atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("d", [0, 1, 2])
def test_collective_reorder_plans_match_torch(dtype, d):
    """The box plans around the collectives (parallel/comm.py _view_boxes): the all-gather send
    buffer (dim d first) and its unpack (blocks into their slices along d, out of group-rank order),
    the reduce-scatter pack (chunks in group-rank order) and the all-to-all pack / unpack — each one
    transfer.hip launch — against the ATen movedim / cat / stack they replace."""
    from flexflow_amd.parallel.comm import _view_boxes
    torch.manual_seed(5)
    k = 4
    x = torch.randn(8, 12, 16, device=DEV).to(dtype)
    order = [2, 0, 3, 1]
    # all-gather: send buffer, then k received blocks unpacked in `order`
    xv = x.movedim(d, 0)
    xm = torch.empty(tuple(xv.shape), device=DEV, dtype=dtype)
    boxcopy.BoxPlan(_view_boxes([(xv, xm)], x, xm), x, xm).run(x, xm)
    assert torch.equal(xm, xv.contiguous())
    out = torch.stack([xm * (i + 1) for i in range(k)], 0).reshape((k * xm.shape[0],) + tuple(xm.shape[1:]))
    chunks = list(out.chunk(k, 0))
    shp = list(x.shape)
    shp[d] *= k
    res = torch.empty(shp, device=DEV, dtype=dtype)
    m0 = xv.shape[0]
    boxcopy.BoxPlan(_view_boxes([(chunks[c].movedim(0, d), res.narrow(d, j * m0, m0)) for j, c in enumerate(order)],
                                out, res), out, res).run(out, res)
    assert torch.equal(res, torch.cat([chunks[c] for c in order], 0).movedim(0, d).contiguous())
    # reduce-scatter pack: x's chunks along d, dim d first, in group-rank order
    if x.shape[d] % k == 0:
        ch = list(xv.chunk(k, 0))
        inp = torch.empty(tuple(xv.shape), device=DEV, dtype=dtype)
        c0 = ch[0].shape[0]
        boxcopy.BoxPlan(_view_boxes([(ch[j], inp.narrow(0, i * c0, c0)) for i, j in enumerate(order)], x, inp),
                        x, inp).run(x, inp)
        assert torch.equal(inp, torch.cat([ch[j] for j in order], 0))
    # all-to-all pack along dim d, unpack along dim (d + 1) % 3
    if x.shape[d] % k == 0:
        a = (d + 1) % 3
        ch = x.chunk(k, dim=d)
        inp = torch.empty((k,) + tuple(ch[0].shape), device=DEV, dtype=dtype)
        boxcopy.BoxPlan(_view_boxes([(ch[order[i]], inp[i]) for i in range(k)], x, inp), x, inp).run(x, inp)
        assert torch.equal(inp, torch.stack([ch[order[i]] for i in range(k)], 0))
        s2 = list(inp.shape[1:])
        s2[a] *= k
        res = torch.empty(s2, device=DEV, dtype=dtype)
        ca = inp.shape[1 + a]
        boxcopy.BoxPlan(_view_boxes([(inp[order[i]], res.narrow(a, i * ca, ca)) for i in range(k)], inp, res),
                        inp, res).run(inp, res)
        assert torch.equal(res, torch.cat([inp[order[i]] for i in range(k)], dim=a))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", ["nhwc_c", "contig_0", "contig_1", "contig_3", "many"])
def test_concat_rows_kernel_matches_torch_cat(dtype, case):
    """Concat forward on transfer.hip's concat_rows (one launch, grid.y = input) against torch.cat:
    Inception's channel-last channel concat, contiguous concats along several dims, 16 inputs;
    widths that do not vectorize fall back (None)."""
    from flexflow_amd.ops.shape import _concat_rows
    torch.manual_seed(6)
    if case == "nhwc_c":
        xs = [torch.randn(8, c, 17, 17, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
              for c in (64, 96, 192, 32)]
        ax = 1
    elif case == "many":
        xs = [torch.randn(5, 8 * (i + 1), device=DEV).to(dtype) for i in range(16)]
        ax = 1
    else:
        ax = int(case[-1])
        base = [6, 10, 4, 8]
        xs = []
        for c in (2, 3, 1):
            s = list(base)
            s[ax] = c * 8 if ax == 3 else c
            xs.append(torch.randn(s, device=DEV).to(dtype))
    out = _concat_rows(xs, ax)
    assert out is not None
    ref = torch.cat(xs, ax)
    assert torch.equal(out, ref)
    if case == "nhwc_c":
        assert out.is_contiguous(memory_format=torch.channels_last)
    odd = [torch.randn(3, 5, device=DEV).to(dtype), torch.randn(3, 7, device=DEV).to(dtype)]
    r = _concat_rows(odd, 1)
    assert r is None or torch.equal(r, torch.cat(odd, 1))


@pytest.mark.parametrize("rows,cols", [(8, 8), (64, 64), (1024, 4096), (3072, 1024), (200, 136), (30528, 1024)])
def test_transpose2d_matches_torch(rows, cols):
    """transpose16 (the Linear layers' W^T copy) against torch's .t(), bitwise; edge tiles included."""
    from flexflow_amd import kernels as Kn
    w = torch.randn(rows, cols, device=DEV).bfloat16()
    out = torch.full((cols, rows), float("nan"), device=DEV, dtype=torch.bfloat16)
    Kn.ext().transpose2d(w, out)
    torch.cuda.synchronize()
    assert torch.equal(out, w.t().contiguous())


@pytest.mark.parametrize("accumulate", [False, True])
def test_linear_bwd_transposed_weight_matches_nn(accumulate):
    """The TN dgrad through weight_t's W^T copy against the NN dgrad and an fp32 torch reference."""
    from flexflow_amd import kernels as Kn
    torch.manual_seed(0)
    M, N, K = 512, 384, 256  # tokens, out, in
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(N, K, device=DEV) / 16).bfloat16()
    dy = torch.randn(M, N, device=DEV).bfloat16()
    store = {}
    wt = Kn.weight_t(store, w)
    assert wt is not None and wt.shape == (K, N)
    base = torch.randn(M, K, device=DEV).bfloat16() if accumulate else None
    outs = []
    for use_wt in (False, True):
        dx_out = base.clone() if accumulate else None
        dw = torch.zeros(N, K, device=DEV)
        dx = Kn.linear_bwd(dy, x, w, None, Kn.ACT_NONE, dw, None, dx_out=dx_out, wt=wt if use_wt else None)
        outs.append((dx.float(), dw))
    torch.cuda.synchronize()
    ref = dy.float() @ w.float() + (base.float() if accumulate else 0)
    for dx, dw in outs:
        assert torch.allclose(dx, ref, atol=3e-2, rtol=2e-2), (dx - ref).abs().max()
        assert torch.allclose(dw, dy.float().t() @ x.float(), atol=5e-2, rtol=1e-2)
    assert torch.allclose(outs[0][0], outs[1][0], atol=3e-2, rtol=2e-2)


def test_transpose2d_batch_matches_torch():
    """One transpose16_batch launch over matrices of different shapes (the executor's per-forward
    W^T refresh) against torch's .t()."""
    from flexflow_amd import kernels as Kn
    shapes = [(1024, 3072), (8, 8), (200, 136), (4096, 1024), (64, 4096)]
    srcs = [torch.randn(r, c, device=DEV).bfloat16() for r, c in shapes]
    stores = []
    for w in srcs:
        st = {}
        Kn.weight_t(st, w)
        st["wt_buf"].fill_(float("nan"))  # the batch must rewrite every element
        stores.append(st)
    cache = {}
    assert Kn.wt_refresh_all(stores, cache) == len(shapes)
    for w in srcs:  # new weight values, same tensors: the cached descriptor table is reused
        w.mul_(-2)
    assert Kn.wt_refresh_all(stores, cache) == len(shapes)
    torch.cuda.synchronize()
    for w, st in zip(srcs, stores):
        assert torch.equal(st["wt_buf"], w.t().contiguous())


def test_bert_losses_with_batched_transposed_weights():
    """A small BERT trained 3 Adam steps with the W^T copies (batched refresh each forward, TN
    dgrads) against the same run with NN dgrads: the losses agree to bf16 summation-order noise."""
    import numpy as np
    from flexflow_amd import kernels as Kn
    from flexflow_amd.core import AdamOptimizer, FFConfig, FFModel, LossType, MetricsType
    from flexflow_amd.models.bert import BertConfig, build_bert

    def run(wt_on):
        Kn._WT["on"] = wt_on
        torch.manual_seed(0)
        cfg = FFConfig(["--dtype", "bf16", "--no-hip-graphs"])
        bc = BertConfig(hidden=256, heads=4, layers=2, ffn=1024, vocab=1024, max_pos=128, seq=128)
        cfg.batch_size = 4
        ff = FFModel(cfg)
        ids, pos, _ = build_bert(ff, 4, bc)
        ff.optimizer = AdamOptimizer(ff, 1e-3)
        ff.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, metrics=[MetricsType.METRICS_ACCURACY])
        rng = np.random.default_rng(0)
        ids.set_tensor(ff, rng.integers(0, bc.vocab, (4, bc.seq), dtype=np.int32))
        pos.set_tensor(ff, np.tile(np.arange(bc.seq, dtype=np.int32), (4, 1)))
        ff.label_tensor.set_tensor(ff, rng.integers(0, bc.vocab, (4, bc.seq, 1), dtype=np.int32))
        losses = []
        for _ in range(3):
            ff.reset_metrics()
            ff.forward()
            ff.zero_gradients()
            ff.backward()
            ff.update()
            losses.append(ff.get_perf_metrics().get_loss())
        torch.cuda.synchronize()
        return np.array(losses)

    try:
        on, off = run(True), run(False)
    finally:
        Kn._WT["on"] = None
    assert np.allclose(on, off, rtol=2e-3), (on, off)
