"""Data structures of the path, mirroring GenomicBreedingCore's ``Genomes``, ``Phenomes`` and
``Fit`` (un-vendored dependency; field usage read from the reference call sites:
src/prediction.jl:53-139 (Genomes/Phenomes fields), src/linear.jl:185-191,232-238 (Fit fields),
src/cross_validation.jl:374-398 (Fit(n, l) placeholder))."""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np


@dataclass
class Genomes:
    """entries x loci-alleles allele frequencies in [0, 1] (NaN = missing)."""
    entries: list
    populations: list
    loci_alleles: list
    allele_frequencies: np.ndarray  # (n, p) float64

    def checkdims(self) -> bool:
        n, p = self.allele_frequencies.shape
        return (len(self.entries) == n and len(self.populations) == n and len(self.loci_alleles) == p
                and len(set(self.entries)) == n and len(set(self.loci_alleles)) == p)


@dataclass
class Phenomes:
    """entries x traits phenotypes (NaN = missing)."""
    entries: list
    populations: list
    traits: list
    phenotypes: np.ndarray  # (n, t) float64

    def checkdims(self) -> bool:
        n, t = self.phenotypes.shape
        return (len(self.entries) == n and len(self.populations) == n and len(self.traits) == t
                and len(set(self.entries)) == n)


@dataclass
class Fit:
    """Model fit; ``b_hat[0]`` is the intercept, ``b_hat_labels[0] == "intercept"`` (src/linear.jl:187)."""
    n: int
    l: int
    model: str = ""
    b_hat_labels: list = field(default_factory=list)
    b_hat: np.ndarray = None
    trait: str = ""
    entries: list = field(default_factory=list)
    populations: list = field(default_factory=list)
    metrics: dict = field(default_factory=dict)
    y_true: np.ndarray = None
    y_pred: np.ndarray = None

    def __post_init__(self):
        if self.b_hat is None:
            self.b_hat = np.zeros(self.l)
        if self.y_true is None:
            self.y_true = np.zeros(self.n)
        if self.y_pred is None:
            self.y_pred = np.zeros(self.n)
        if not self.b_hat_labels:
            self.b_hat_labels = [""] * self.l
        if not self.entries:
            self.entries = [""] * self.n
        if not self.populations:
            self.populations = [""] * self.n

    def checkdims(self) -> bool:
        # `l` is only the initial allocation: ridge re-assigns a (p+1)-long b_hat after
        # Fit(n, l=p) (src/linear.jl:185,232), so consistency is between the fields themselves.
        n = len(self.entries)
        return (len(self.b_hat) == len(self.b_hat_labels) and n == self.n
                and len(self.populations) == self.n and len(self.y_true) == self.n and len(self.y_pred) == self.n)
