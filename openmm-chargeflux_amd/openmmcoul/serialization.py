"""XML serialization of CoulForce (the reference registers no
SerializationProxy, so a System holding this force cannot be saved or reloaded).

The document is the one OpenMM's ``XmlSerializer`` writes for a force with the plugin's C++
``CoulForceProxy`` (openmm-chargeflux_amd/plugin/src/CoulForceProxy.cpp): root element ``Force``
with ``type="CoulForce"`` and a ``version``, parameters as attributes, one child list per kind
of entry (tests/test_plugin_openmm.py reads each side's output with the other):

    <Force type="CoulForce" version="1" forceGroup="0" cutoff="1.0" ewaldTolerance="0.0001" usesPeriodic="1">
      <Particles>   <Particle q=".." sig=".." eps=".."/> ...           CoulForce.cpp:18-38
      <Exceptions>  <Exception p1=".." p2=".."/> ...                   CoulForce.cpp:56-68
      <FluxBonds>   <FluxBond p1 p2 k b/> ...                          CoulForce.cpp:78-94
      <FluxAngles>  <FluxAngle p1 p2 p3 k theta/> ...                  CoulForce.cpp:96-114
      <FluxWaters>  <FluxWater po ph1 ph2 k1 k2 kub b0 ub0/> ...       CoulForce.cpp:116-140
    </Force>

Floats are written with ``repr`` (shortest round-trip form; the C++ proxy writes 17 significant
digits), so either reader reproduces every parameter bit for bit.  The round-2 form of this
file, root element ``<CoulForce ...>`` without ``type``, is still read.
"""
from __future__ import annotations

import xml.etree.ElementTree as ET

from .force import CoulForce

VERSION = 1


def _f(x: float) -> str:
    return repr(float(x))


class XmlSerializer:
    """serialize(CoulForce) -> str and deserialize(str) -> CoulForce (OpenMM's
    XmlSerializer.serialize / deserialize names)."""

    @staticmethod
    def serialize(force: CoulForce) -> str:
        if not isinstance(force, CoulForce):
            raise TypeError("XmlSerializer.serialize expects a CoulForce")
        root = ET.Element("Force", {
            "type": "CoulForce",
            "version": str(VERSION),
            "forceGroup": str(force.getForceGroup()),
            "cutoff": _f(force.getCutoffDistance()),
            "ewaldTolerance": _f(force.getEwaldErrorTolerance()),
            "usesPeriodic": "1" if force.usesPeriodicBoundaryConditions() else "0",
        })
        parts = ET.SubElement(root, "Particles")
        for i in range(force.getNumParticles()):
            q, sig, eps = force.getParticleParameters(i)
            ET.SubElement(parts, "Particle", {"q": _f(q), "sig": _f(sig), "eps": _f(eps)})
        exc = ET.SubElement(root, "Exceptions")
        for k in range(force.getNumExceptions()):
            p1, p2 = force.getExceptionParameters(k)
            ET.SubElement(exc, "Exception", {"p1": str(p1), "p2": str(p2)})
        fb = ET.SubElement(root, "FluxBonds")
        for k in range(force.getNumFluxBonds()):
            p1, p2, kk, b = force.getFluxBondParameters(k)
            ET.SubElement(fb, "FluxBond", {"p1": str(p1), "p2": str(p2), "k": _f(kk), "b": _f(b)})
        fa = ET.SubElement(root, "FluxAngles")
        for k in range(force.getNumFluxAngles()):
            p1, p2, p3, kk, th = force.getFluxAngleParameters(k)
            ET.SubElement(fa, "FluxAngle", {"p1": str(p1), "p2": str(p2), "p3": str(p3), "k": _f(kk),
                                            "theta": _f(th)})
        fw = ET.SubElement(root, "FluxWaters")
        for k in range(force.getNumFluxWaters()):
            po, h1, h2, k1, k2, kub, b0, ub0 = force.getFluxWaterParameters(k)
            ET.SubElement(fw, "FluxWater", {"po": str(po), "ph1": str(h1), "ph2": str(h2), "k1": _f(k1),
                                            "k2": _f(k2), "kub": _f(kub), "b0": _f(b0), "ub0": _f(ub0)})
        ET.indent(root)
        return ET.tostring(root, encoding="unicode") + "\n"

    @staticmethod
    def deserialize(text: str) -> CoulForce:
        root = ET.fromstring(text)
        if not (root.tag == "CoulForce" or root.get("type") == "CoulForce"):
            raise ValueError(f"not a CoulForce document (root element <{root.tag}>, type {root.get('type')!r})")
        version = int(root.get("version", "0"))
        if version < 1 or version > VERSION:
            raise ValueError(f"unsupported CoulForce serialization version {version}")
        f = CoulForce()
        f.setForceGroup(int(root.get("forceGroup", "0")))
        f.setCutoffDistance(float(root.get("cutoff")))
        f.setEwaldErrorTolerance(float(root.get("ewaldTolerance")))
        f.setUsesPeriodicBoundaryConditions(root.get("usesPeriodic") == "1")

        def items(group, tag):
            g = root.find(group)
            return [] if g is None else g.findall(tag)

        for e in items("Particles", "Particle"):
            f.addParticle(float(e.get("q")), float(e.get("sig")), float(e.get("eps")))
        for e in items("Exceptions", "Exception"):
            f.addException(int(e.get("p1")), int(e.get("p2")))
        for e in items("FluxBonds", "FluxBond"):
            f.addFluxBond(int(e.get("p1")), int(e.get("p2")), float(e.get("k")), float(e.get("b")))
        for e in items("FluxAngles", "FluxAngle"):
            f.addFluxAngle(int(e.get("p1")), int(e.get("p2")), int(e.get("p3")), float(e.get("k")),
                           float(e.get("theta")))
        for e in items("FluxWaters", "FluxWater"):
            f.addFluxWater(int(e.get("po")), int(e.get("ph1")), int(e.get("ph2")), float(e.get("k1")),
                           float(e.get("k2")), float(e.get("kub")), float(e.get("b0")), float(e.get("ub0")))
        n = f.getNumParticles()
        for k in range(f.getNumExceptions()):
            for a in f.getExceptionParameters(k):
                if not 0 <= a < n:
                    raise ValueError(f"exception {k} refers to particle {a} of {n}")
        return f
