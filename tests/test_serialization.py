"""XML serialization of CoulForce (the reference has no proxy): exact
round trip of every parameter, version checks, and that a deserialized force gives the same
oracle energy as the original.  CPU only."""
import numpy as np
import pytest

from oracle import Oracle
from openmmcoul import CoulForce, XmlSerializer
from openmmcoul import testsystems as ts


def _same(a: CoulForce, b: CoulForce):
    assert a.getNumParticles() == b.getNumParticles()
    assert a.getCutoffDistance() == b.getCutoffDistance()
    assert a.getEwaldErrorTolerance() == b.getEwaldErrorTolerance()
    assert a.usesPeriodicBoundaryConditions() == b.usesPeriodicBoundaryConditions()
    assert a.getForceGroup() == b.getForceGroup()
    for k, v in a.arrays().items():
        w = b.arrays()[k]
        assert v.shape == w.shape, k
        assert np.array_equal(v, w), k   # bit-exact (repr round trip)


@pytest.mark.parametrize("which", ["C1", "box"])
def test_round_trip_exact(which):
    if which == "C1":
        _, f, _, _ = ts.cluster_c1()
    else:
        _, f, _, _ = ts.water_box(60, cutoff=0.6, every_bond_angle=3)
    # awkward floats survive
    f.setParticleParameters(0, 0.1 + 0.2, 1.0 / 3.0, 2.0 ** -40)
    f.setForceGroup(5)
    text = XmlSerializer.serialize(f)
    assert text.startswith('<Force type="CoulForce"') and 'version="1"' in text
    g = XmlSerializer.deserialize(text)
    _same(f, g)
    assert XmlSerializer.serialize(g) == text


def test_empty_force_and_errors():
    f = CoulForce()
    g = XmlSerializer.deserialize(XmlSerializer.serialize(f))
    _same(f, g)
    with pytest.raises(ValueError):
        XmlSerializer.deserialize("<NonbondedForce version='1'/>")
    with pytest.raises(ValueError):
        XmlSerializer.deserialize("<Force type='NonbondedForce' version='1'/>")
    # the round-2 root element is still read
    legacy = XmlSerializer.serialize(f).replace('<Force type="CoulForce"', "<CoulForce").replace("</Force>", "</CoulForce>")
    _same(f, XmlSerializer.deserialize(legacy))
    with pytest.raises(ValueError):
        XmlSerializer.deserialize("<CoulForce version='99' cutoff='1' ewaldTolerance='1e-4' usesPeriodic='0'/>")
    with pytest.raises(TypeError):
        XmlSerializer.serialize(object())
    bad = ("<CoulForce version='1' cutoff='1' ewaldTolerance='1e-4' usesPeriodic='0'>"
           "<Particles><Particle q='1' sig='0' eps='0'/></Particles>"
           "<Exceptions><Exception p1='0' p2='3'/></Exceptions></CoulForce>")
    with pytest.raises(ValueError):
        XmlSerializer.deserialize(bad)


def test_deserialized_force_evaluates_identically():
    _, f, pos, box = ts.water_box(40, cutoff=0.5, ewald_tol=1e-4, every_bond_angle=2)
    g = XmlSerializer.deserialize(XmlSerializer.serialize(f))
    a = Oracle(f, box).execute(pos, box)
    b = Oracle(g, box).execute(pos, box)
    assert a["energy"] == b["energy"]
    assert np.array_equal(a["forces"], b["forces"])
