"""Wavelet filter banks (the DATA side of jwave/transforms/wavelets/).

Tap values live in ``data/taps.json``, evaluated from the reference's wavelet
constructors by ``tools/gen_taps.py`` (bit-identical doubles).  A ``Wavelet``
exposes the getters the engine needs (Wavelet.java:152-219); the kernel math
itself lives in libjwave_hip.so.
"""
import json
import os

from .exceptions import JWaveFailure

_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "taps.json")
_DB = None


def _db():
    global _DB
    if _DB is None:
        with open(_DATA) as fh:
            _DB = json.load(fh)
    return _DB


class Wavelet:
    """A discrete wavelet's filter bank (mirror of jwave.transforms.wavelets.Wavelet)."""

    def __init__(self, rec):
        self.cls = rec["class"]
        self.name = rec["name"]
        self.mother_wavelength = int(rec["mother_wavelength"])
        self.transform_wavelength = int(rec["transform_wavelength"])
        self.lo = list(map(float, rec["lo"]))
        self.hi = list(map(float, rec["hi"]))
        self.lo_r = list(map(float, rec["lo_r"]))
        self.hi_r = list(map(float, rec["hi_r"]))
        self.reverse_scale = float(rec["reverse_scale"])
        self.source = rec.get("source", "")

    # reference getter names (Wavelet.java:128-219)
    def getName(self):  # noqa: N802
        return self.name

    def getMotherWavelength(self):  # noqa: N802
        return self.mother_wavelength

    def getTransformWavelength(self):  # noqa: N802
        return self.transform_wavelength

    def getScalingDeComposition(self):  # noqa: N802
        return list(self.lo)

    def getWaveletDeComposition(self):  # noqa: N802
        return list(self.hi)

    def getScalingReConstruction(self):  # noqa: N802
        return list(self.lo_r)

    def getWaveletReConstruction(self):  # noqa: N802
        return list(self.hi_r)

    def __repr__(self):
        return "Wavelet(%s, L=%d)" % (self.name, self.mother_wavelength)

    def __str__(self):
        return self.name


def by_class(cls):
    """Wavelet by reference class name, e.g. ``by_class("Daubechies4")``."""
    recs = _db()["wavelets"]
    if cls not in recs:
        raise KeyError(cls)
    return Wavelet(recs[cls])


def class_names():
    return sorted(_db()["wavelets"])


class WaveletBuilder:
    """Name -> Wavelet factory (WaveletBuilder.java:99-409, create2arr :427-502)."""

    @staticmethod
    def create(name):
        db = _db()
        if name in db["builder_refuses"]:
            # WaveletBuilder.java:363-385: odd tap counts are refused
            raise JWaveFailure("WaveletBuilder::create - " + name.replace(" ", "") +
                               " - This wavelet has an odd number of coefficients, due to that it"
                               " is not comaptible to the implemented algorithms; somehow!")
        cls = db["builder_names"].get(name)
        if cls is None:
            raise JWaveFailure("WaveletBuilder::create - unknown type of wavelet for given string!")
        return by_class(cls)

    @staticmethod
    def create2arr():
        return [WaveletBuilder.create(n) for n in _db()["create2arr"]]


def __getattr__(name):  # jwave_amd.wavelets.Daubechies4() style constructors
    if name in _db()["wavelets"]:
        return lambda: by_class(name)
    raise AttributeError(name)
