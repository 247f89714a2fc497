"""leading_relu_branch_{combine,partition} (reference substitution.cc:3463-3540, generated for
num_combines 1..4 at substitution.cc:1839-1841): matched on the forks of Inception, applied as
sample-degree pins on the fork's branches, and rebuilt from their names on another process."""
from flexflow_amd.core import FFConfig, FFModel
from flexflow_amd.models import build
from flexflow_amd.pcg import joint


def _inception(workers=4):
    cfg = FFConfig(["--search-num-workers", str(workers)])
    cfg.batch_size = 8
    ff = FFModel(cfg)
    build("inception_v3", ff, 8, small=True)
    return ff


def _readers(ff):
    r = {}
    for L in ff.layers:
        for t in L.inputs:
            r.setdefault(t.guid, []).append(L)
    return r


def test_generated_for_every_degree_and_branch_count():
    ff = _inception(4)
    names = {x.name for x in joint.build_xfers(ff) if isinstance(x, joint.LeadingBranch)}
    for d in (2, 4):
        for num in range(1, 5):
            assert f"leading_relu_branch_combine[{d},{num}]" in names
            assert f"leading_relu_branch_partition[{d},{num}]" in names


def test_combine_pins_leading_branch_and_siblings():
    ff = _inception(4)
    x = joint.LeadingBranch("leading_relu_branch_combine", 2, 2)
    ms = x.matches(ff)
    assert ms
    _, d, num, positions = ms[0]
    olds = [ff.layers[p] for p in positions]
    # the pinned ops are the first num + 1 readers of one fork tensor
    shared = set.intersection(*[{t.guid for t in L.inputs} for L in olds])
    assert shared and len(olds) == num + 1
    assert x.apply(ff, ms[0])
    pinned = [L for L in ff.layers if "pin" in L.attrs]
    assert len(pinned) == num + 1
    assert all(L.attrs["pin"][0] == d and all(v == 1 for v in L.attrs["pin"][1:]) for L in pinned)


def test_partition_pins_producer_and_siblings_not_leader():
    ff = _inception(4)
    x = joint.LeadingBranch("leading_relu_branch_partition", 2, 1)
    ms = x.matches(ff)
    assert ms
    positions = ms[0][3]
    prod, sib = ff.layers[positions[0]], ff.layers[positions[1]]
    readers = _readers(ff)[prod.outputs[0].guid]
    assert sib in readers and readers[0] is not sib  # the leading branch stays free
    assert x.apply(ff, ms[0])
    assert sorted(L.name.split("@")[0] for L in ff.layers if "pin" in L.attrs) == sorted([prod.name, sib.name])


def test_replays_from_its_name_on_a_fresh_graph():
    ff = _inception(4)
    x = joint.LeadingBranch("leading_relu_branch_partition", 2, 2)
    m = x.matches(ff)[0]
    assert x.apply(ff, m)

    def shape(model):  # layer names carry a process-wide counter: compare kinds and pins
        return [(L.op_type.value, L.attrs.get("pin")) for L in model.layers]

    ff2 = _inception(1)  # a process whose machine would not generate degree-2 xfers itself
    joint.replay(ff2, [], [(x.name, m)])
    assert shape(ff2) == shape(ff) and sum(1 for L in ff2.layers if "pin" in L.attrs) == 3
