"""The one-launch training step (csrc/train_dag.hip) against the
launch-per-GEMM step, on the MI355X.

The persistent kernel runs the step's job DAG -- input preparation, every GEMM tile of the
launch path (with its epilogues and the k-group split of the launch's tile), the bias sums and
every AdamW tile -- so it must reproduce the launch path BIT FOR BIT: losses, fp32 masters,
Adam moments, both bf16 working copies and the gradients.  That path is itself pinned to the
fp64 oracle (test_gpu_train_capi.py, test_gpu_configs.py::test_config2_*)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import ldm_sdf
    ldm_sdf.load_library()
    return torch.device("cuda", 0)


@pytest.fixture
def form():
    """Set the training-step form for one test and restore the default afterwards."""
    from ldm_sdf import ops
    yield ops.train_step_config
    ops.train_step_config("auto")


def _run(dev, form_name, *, D=256, H=1024, nb=4, TE=128, M=300, batch=None, steps=6,
         graph=False, seed=11):
    import ldm_sdf
    from ldm_sdf import MLPDenoiser, ops
    ops.train_step_config(form_name)
    model = MLPDenoiser(D=D, H=H, n_blocks=nb, TE=TE, seed=seed)
    model.to_device(dev)
    sch = ldm_sdf.DDPMSchedule()
    lat = torch.randn(M, D, generator=torch.Generator().manual_seed(5)).to(dev) * 0.5
    gen = torch.Generator(device=dev).manual_seed(3)
    st = ldm_sdf.train(model, sch, lat, steps=steps, batch=batch or M, lr=1e-3,
                       weight_decay=0.01, dtype="bf16", generator=gen, graph=graph)
    last = ops.train_step_last_form()
    work = model.device_pack("bf16", dev, with_tables=False)
    torch.cuda.synchronize()
    return (last, list(st.losses), {n: t.clone() for n, t in model.params.items()},
            {n: (m.clone(), v.clone()) for n, (m, v) in st.adam.items()},
            {n: t.clone() for n, t in work.items() if isinstance(t, torch.Tensor)},
            {n: g.clone() for n, g in st.adam_grads.items()})


def _assert_same(a, b):
    assert a[1] == b[1], (a[1], b[1])                        # losses
    for n in b[2]:
        assert torch.equal(a[2][n], b[2][n]), ("master", n)
        assert torch.equal(a[3][n][0], b[3][n][0]) and torch.equal(a[3][n][1], b[3][n][1]), n
        assert torch.equal(a[5][n], b[5][n]), ("grad", n)
    for n in b[4]:
        assert torch.equal(a[4][n], b[4][n]), ("working copy", n)


@pytest.mark.parametrize("M", [1000, 300, 37])
def test_dag_step_bitwise_vs_launches(dev, form, M):
    """Config 2's shape (batch 1000 = 16 row bands, the last one ragged), a mid batch and a
    one-band batch: 6 steps of train() through the DAG == through the launches, bit for bit."""
    ref = _run(dev, "launches", M=M)
    got = _run(dev, "dag", M=M)
    assert ref[0] == "launches" and got[0] == "dag"
    _assert_same(got, ref)


@pytest.mark.parametrize("nb,H,D,TE", [(1, 256, 128, 64), (2, 512, 64, 128), (8, 256, 256, 64)])
def test_dag_other_networks_bitwise(dev, form, nb, H, D, TE):
    """The DAG is built from the recorded launches, so other depths / widths (1, 2 and 8
    residual blocks) reproduce the launch path too."""
    ref = _run(dev, "launches", D=D, H=H, nb=nb, TE=TE, M=200, steps=4)
    got = _run(dev, "dag", D=D, H=H, nb=nb, TE=TE, M=200, steps=4)
    assert got[0] == "dag"
    _assert_same(got, ref)


def test_dag_graph_replay_bitwise(dev, form):
    """train(graph=True) replays hipGraphs of the one-launch step (t, eps and the AdamW scalars
    refilled per 32-step block): bit-identical to the eager DAG steps over 40 steps."""
    ref = _run(dev, "dag", M=256, steps=40)
    got = _run(dev, "dag", M=256, steps=40, graph=True)
    assert got[0] == "dag"
    _assert_same(got, ref)


def test_dag_timeout_surfaces_then_recovers(dev, form):
    """A dependency wait that gives up (spin limit 1 us) raises the status word, every
    workgroup drains and exits, and train() reports it (LdmError); the next run (default limit)
    starts from zeroed counters and matches the launch path again."""
    import ldm_sdf
    from ldm_sdf import LdmError, MLPDenoiser, ops
    model = MLPDenoiser(seed=11)
    model.to_device(dev)
    sch = ldm_sdf.DDPMSchedule()
    lat = torch.randn(300, 256, generator=torch.Generator().manual_seed(5)).to(dev) * 0.5
    ops.train_step_config("dag", spin_limit=1)
    with pytest.raises(LdmError, match="status 1"):
        ldm_sdf.train(model, sch, lat, steps=3, batch=300, dtype="bf16")
    ref = _run(dev, "launches", M=300, steps=3)
    got = _run(dev, "dag", M=300, steps=3)
    _assert_same(got, ref)


def test_dag_required_form_fails_loudly_with_side_stream(dev, form):
    """form "dag" with a side stream (the overlap option, which the one-launch step has no use
    for) is refused with LDM_ENOSYS, not run silently on the launch path; "auto" with a side
    stream runs the launches."""
    import ldm_sdf
    from ldm_sdf import LdmError, MLPDenoiser, ops
    model = MLPDenoiser(seed=11)
    model.to_device(dev)
    lat = torch.randn(64, 256, generator=torch.Generator().manual_seed(5)).to(dev) * 0.5
    ops.train_step_config("dag")
    ldm_sdf.train(model, ldm_sdf.DDPMSchedule(), lat, steps=1, batch=64, dtype="bf16")
    assert ops.train_step_last_form() == "dag"
    with pytest.raises(LdmError):
        ldm_sdf.train(model, ldm_sdf.DDPMSchedule(), lat, steps=1, batch=64, dtype="bf16",
                      overlap=True)
    ops.train_step_config("auto")
    ldm_sdf.train(model, ldm_sdf.DDPMSchedule(), lat, steps=1, batch=64, dtype="bf16",
                  overlap=True)
    assert ops.train_step_last_form() == "launches"


def _dag_flags(v):
    import ctypes as C
    from ldm_sdf import _capi as capi
    fl = getattr(capi.load(), "ldm_dev_train_dag_flags", None)
    if fl is None:
        pytest.skip("ldm_dev_train_dag_flags is exported by the development build only "
                    "(make DEV=1); the product library has no diagnostic switches")
    fl.restype, fl.argtypes = C.c_int, [C.c_uint]
    return fl(v)


@pytest.mark.parametrize("flags", [0x100, 0x200])
@pytest.mark.parametrize("M", [1000, 37])
def test_dag_claim_scheduler_bitwise(dev, form, M, flags):
    """The claim scheduler (0x100: a workgroup takes only READY jobs, chain list first;
    train_dag.hip, kDbgClaim) and the weight operands loaded through the L2 (0x200,
    kDbgWeightsL2) compute the same step bit for bit: neither changes an arithmetic.
    (Development build only: skipped against the product library.)"""
    _dag_flags(0)
    ref = _run(dev, "launches", M=M)
    _dag_flags(flags)
    try:
        got = _run(dev, "dag", M=M)
    finally:
        _dag_flags(0)
    assert got[0] == "dag"
    _assert_same(got, ref)


def test_trainstate_save_resume_bitwise(dev, tmp_path):
    """SURVEY §5 checkpoint / resume: 64 uninterrupted steps == 32 steps, TrainState.save
    (masters, AdamW moments, step, losses, generator state), a FRESH denoiser object loading it
    (TrainState.load), 32 more steps -- bit for bit: losses, masters, moments."""
    import ldm_sdf
    from ldm_sdf import MLPDenoiser
    from ldm_sdf.api import TrainState
    sch = ldm_sdf.DDPMSchedule()
    lat = torch.randn(256, 256, generator=torch.Generator().manual_seed(5)).to(dev) * 0.5

    def fresh(seed):
        m = MLPDenoiser(seed=seed)
        m.to_device(dev)
        return m

    ref = fresh(11)
    g = torch.Generator(device=dev).manual_seed(3)
    st = ldm_sdf.train(ref, sch, lat, steps=64, batch=256, lr=1e-3, weight_decay=0.01,
                       dtype="bf16", generator=g)
    a = fresh(11)
    g2 = torch.Generator(device=dev).manual_seed(3)
    st_a = ldm_sdf.train(a, sch, lat, steps=32, batch=256, lr=1e-3, weight_decay=0.01,
                         dtype="bf16", generator=g2)
    path = str(tmp_path / "train_state.pt")
    st_a.save(path, generator=g2)
    b = fresh(999)                               # other weights: all must come from the file
    g3 = torch.Generator(device=dev).manual_seed(12345)
    st_b = TrainState.load(path, b, device=dev, generator=g3)
    assert st_b.step == 32 and st_b.hparams == {"lr": 1e-3, "weight_decay": 0.01}
    st_b = ldm_sdf.train(b, sch, lat, steps=32, batch=256, dtype="bf16", generator=g3,
                         state=st_b)
    torch.cuda.synchronize()
    assert st_b.step == 64
    assert st_b.losses == st.losses
    for n in ref.params:
        assert torch.equal(b.params[n], ref.params[n]), n
        assert torch.equal(st_b.adam[n][0], st.adam[n][0]) and \
            torch.equal(st_b.adam[n][1], st.adam[n][1]), n
    # and the resumed model samples like the uninterrupted one
    xT = torch.randn(4, 256, generator=torch.Generator().manual_seed(1)).to(dev)
    nz = torch.randn(1000, 4, 256, generator=torch.Generator().manual_seed(2)).to(dev)
    s_ref = ldm_sdf.sample(ref, sch, 4, steps=20, x_T=xT, noise=nz, device=dev)
    s_b = ldm_sdf.sample(b, sch, 4, steps=20, x_T=xT, noise=nz, device=dev)
    assert torch.equal(s_ref, s_b)


def test_trainstate_resume_with_torch_optimizer_bitwise(dev, tmp_path):
    """a caller's torch optimizer built on a fresh denoiser's parameters BEFORE
    TrainState.load must, after the load, update the loaded masters (the tensors train()
    trains), not the replaced ones.  32 steps == 32 + save + load + 32 more, bit for bit, with
    torch.optim.AdamW on both sides (losses and parameters)."""
    import ldm_sdf
    from ldm_sdf import MLPDenoiser
    from ldm_sdf.api import TrainState
    sch = ldm_sdf.DDPMSchedule()
    lat = torch.randn(256, 256, generator=torch.Generator().manual_seed(5)).to(dev) * 0.5

    def fresh(seed):
        m = MLPDenoiser(seed=seed)
        m.to_device(dev)
        return m

    def torch_state(m):
        st = TrainState()
        st.masters = {n: m.params[n] for n in m.names()}
        st.optimizer = torch.optim.AdamW(list(st.masters.values()), lr=1e-3, weight_decay=0.01)
        return st

    ref = fresh(11)
    g = torch.Generator(device=dev).manual_seed(3)
    st = ldm_sdf.train(ref, sch, lat, steps=64, batch=256, dtype="bf16", generator=g,
                       state=torch_state(ref))
    a = fresh(11)
    g2 = torch.Generator(device=dev).manual_seed(3)
    st_a = ldm_sdf.train(a, sch, lat, steps=32, batch=256, dtype="bf16", generator=g2,
                         state=torch_state(a))
    path = str(tmp_path / "train_state_opt.pt")
    st_a.save(path, generator=g2)
    b = fresh(999)
    opt_b = torch.optim.AdamW(list(b.params.values()), lr=1e-3, weight_decay=0.01)
    g3 = torch.Generator(device=dev).manual_seed(12345)
    st_b = TrainState.load(path, b, device=dev, generator=g3, optimizer=opt_b)
    assert {id(p) for p in opt_b.param_groups[0]["params"]} == \
        {id(t) for t in st_b.masters.values()}
    st_b = ldm_sdf.train(b, sch, lat, steps=32, batch=256, dtype="bf16", generator=g3,
                         state=st_b)
    torch.cuda.synchronize()
    assert st_b.losses == st.losses
    for n in ref.params:
        assert torch.equal(b.params[n], ref.params[n]), n
