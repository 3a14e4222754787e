"""The GRM arithmetic as a per-call argument of the drop-in boundary (include/gbm.h GBM_GRM_*, the _ex entries;
Julia `gblup(...; grm = :auto)`). The reference hands gblup the allele-frequency matrix of extractxyetc
(src/prediction.jl:129); for diploids those are dosages/2, and `auto` must route such X to the exact-integer GRM
(csrc/grm_exact.hip) and every other X to the fp64-MFMA SYRK — both against the oracle (src/gwas.jl:112-126,
591-597 restated in oracle/oracle.py). GBM_GRM only supplies the mode of calls that pass GBM_GRM_DEFAULT."""
import numpy as np
import pytest

import gbm
import oracle
from gbm.types import Genomes, Phenomes

pytestmark = pytest.mark.gpu

TOL_Y, TOL_B = 1e-9, 1e-6


def rel(a, b):
    return float(np.abs(np.asarray(a) - np.asarray(b)).max() / np.abs(np.asarray(b)).max())


def check(out, ref):
    b, y, mu, q = out
    assert q == ref["q"] and rel(y, ref["y_pred"]) < TOL_Y and rel(mu, ref["mu"]) < TOL_Y
    assert rel(b, ref["b_hat"]) < TOL_B


@pytest.fixture(scope="module")
def dosage_case():
    n, p = 777, 2345
    X = oracle.synth_genotypes(31, n, p)  # dosage / 2
    Y = oracle.synth_phenotypes(X, 32, ntraits=2)
    return X, Y, oracle.gblup_fit(X, Y, 1.0)


def test_auto_routes_dosage_x_to_exact(dosage_case):
    X, Y, ref = dosage_case
    info = {}
    out = gbm.gblup_arrays(X, Y, grm="auto", info=info)
    assert info["grm_used"] == "exact"
    check(out, ref)
    info_e = {}
    ex = gbm.gblup_arrays(X, Y, grm="exact", info=info_e)
    assert info_e["grm_used"] == "exact"
    for a, b in zip(ex, out):
        assert np.array_equal(np.asarray(a), np.asarray(b))
    info_f = {}
    fp = gbm.gblup_arrays(X, Y, grm="fp64", info=info_f)
    assert info_f["grm_used"] == "fp64"
    check(fp, ref)


def test_auto_routes_other_x_to_fp64(dosage_case):
    X, Y, _ = dosage_case
    n, p = X.shape
    cases = {
        "frequencies": np.clip(X + np.random.default_rng(5).normal(0, 0.01, X.shape), 0, 1),  # imputed values
        "tetraploid": np.rint(X * 4 * 0.75) / 4,  # dosages/4 with odd dosages: 2x = 0.5, 1.5 occur
        "last_locus_only": X.copy(),  # dosage-valued except one cell of the last locus (after the first chunk)
    }
    cases["last_locus_only"][n // 2, p - 1] = 0.3
    for name, Xc in cases.items():
        ref = oracle.gblup_fit(Xc, Y, 1.0)
        info = {}
        out = gbm.gblup_arrays(Xc, Y, grm="auto", info=info)
        assert info["grm_used"] == "fp64", name
        check(out, ref)
        with pytest.raises(gbm.ArgumentError, match="not diploid dosages"):
            gbm.gblup_arrays(Xc, Y, grm="exact")


def test_auto_multi_shard_and_reml(dosage_case):
    X, Y, ref = dosage_case
    info = {}
    out = gbm.gblup_arrays(X, Y, grm="auto", devices=[0, 0, 0], info=info)
    assert info["grm_used"] == "exact"
    check(out, ref)
    info = {}
    b, y, mu, q, r = gbm.gblup_reml_arrays(X, Y[:, 0], grm="auto", info=info)
    b2, y2, mu2, q2, r2 = gbm.gblup_reml_arrays(X, Y[:, 0], grm="fp64")
    assert info["grm_used"] == "exact"
    assert abs(r["lambda"][0] - r2["lambda"][0]) < 1e-6 * r2["lambda"][0] and rel(y, y2) < 1e-8


def test_int8_and_synthetic_sources():
    n, p = 640, 1500
    X = oracle.synth_genotypes(41, n, p)
    Y = oracle.synth_phenotypes(X, 42, ntraits=1)
    ref = oracle.gblup_fit(X, Y, 1.0)
    D = np.rint(2 * X).astype(np.int8)
    info = {}
    check(gbm.gblup_dosage(D, 2, Y, grm="auto", info=info), ref)
    assert info["grm_used"] == "exact"
    info = {}
    check(gbm.gblup_synthetic(41, n, p, Y, grm="auto", info=info), ref)
    assert info["grm_used"] == "exact"
    # tetraploid bytes: auto keeps fp64, exact refuses before any device work
    D4 = np.rint(4 * X * 0.75).astype(np.int8)
    ref4 = oracle.gblup_fit(D4 / 4.0, Y, 1.0)
    info = {}
    check(gbm.gblup_dosage(D4, 4, Y, grm="auto", info=info), ref4)
    assert info["grm_used"] == "fp64"
    # a byte outside {0, 1, 2} at ploidy 2: auto falls back to fp64 (x = 1.5 is a valid frequency), exact refuses
    Db = D.copy()
    Db[3, p - 2] = 3
    refb = oracle.gblup_fit(Db / 2.0, Y, 1.0)
    info = {}
    check(gbm.gblup_dosage(Db, 2, Y, grm="auto", info=info), refb)
    assert info["grm_used"] == "fp64"
    with pytest.raises(gbm.ArgumentError, match="outside"):
        gbm.gblup_dosage(Db, 2, Y, grm="exact")


def test_environment_only_supplies_the_default(dosage_case, gbm_env):
    X, Y, ref = dosage_case
    gbm_env.setenv("GBM_GRM", "exact")
    info = {}
    check(gbm.gblup_arrays(X, Y, grm="fp64", info=info), ref)
    assert info["grm_used"] == "fp64"  # the argument wins
    info = {}
    check(gbm.gblup_arrays(X, Y, grm=None, info=info), ref)
    assert info["grm_used"] == "exact"  # GBM_GRM_DEFAULT: the environment
    gbm_env.delenv("GBM_GRM")
    info = {}
    gbm.gblup_arrays(X, Y, grm=None, info=info)
    assert info["grm_used"] == "fp64"


def test_dropin_default_follows_a_set_grm_variable(dosage_case, gbm_env):
    """The drop-in's default (grm="dropin", Julia grm = :dropin): GBM_GRM=fp64 set by a user or CI
    pins the fp64 SYRK for gblup as for every other entry; unset, the drop-in is auto (exact on dosages)."""
    X, Y, ref = dosage_case
    n, p = X.shape
    genomes = Genomes(entries=[f"e{i}" for i in range(n)], populations=["pop"] * n,
                      loci_alleles=[f"chr1\t{j}\tA|T\tA" for j in range(p)], allele_frequencies=X)
    phenomes = Phenomes(entries=genomes.entries, populations=genomes.populations, traits=["t1"],
                        phenotypes=Y[:, :1].copy())
    gbm_env.setenv("GBM_GRM", "fp64")
    assert gbm.gblup(genomes=genomes, phenomes=phenomes).grm_used == "fp64"
    assert gbm.gblup(genomes=genomes, phenomes=phenomes, grm="auto").grm_used == "exact"  # an argument wins
    gbm_env.setenv("GBM_GRM", "exact")
    assert gbm.gblup(genomes=genomes, phenomes=phenomes).grm_used == "exact"
    gbm_env.delenv("GBM_GRM")
    fit = gbm.gblup(genomes=genomes, phenomes=phenomes)
    assert fit.grm_used == "exact"
    assert rel(fit.y_pred, ref["y_pred"][:, 0]) < 1e-9


def test_model_function_default_auto_and_sessions(dosage_case):
    """The drop-in gblup (grm="dropin" by default: auto with GBM_GRM unset) records the GRM it used; a session of
    fp64 X checks once whether its genotypes are dosages/2 and builds exact training GRMs under auto."""
    X, Y, _ = dosage_case
    n, p = X.shape
    genomes = Genomes(entries=[f"e{i}" for i in range(n)], populations=["pop"] * n,
                      loci_alleles=[f"chr1\t{j}\tA|T\tA" for j in range(p)], allele_frequencies=X)
    phenomes = Phenomes(entries=genomes.entries, populations=genomes.populations, traits=["t1"],
                        phenotypes=Y[:, :1].copy())
    fit = gbm.gblup(genomes=genomes, phenomes=phenomes)
    assert fit.grm_used == "exact"
    fit64 = gbm.gblup(genomes=genomes, phenomes=phenomes, grm="fp64")
    assert fit64.grm_used == "fp64" and rel(fit.y_pred, fit64.y_pred) < 1e-9
    from gbm.session import GenotypeSession
    idx = np.arange(0, n, 2)
    ref = oracle.gblup_fit(np.asfortranarray(X[idx]), Y[idx], 1.0)
    with GenotypeSession(X) as s:
        s.set_grm("auto")
        check(s.gblup(idx, Y[idx]), ref)
        assert s.grm_used() == "exact"
        s.set_grm("fp64")  # the cache is keyed by the GRM used: rebuilt in fp64
        check(s.gblup(idx, Y[idx]), ref)
        assert s.grm_used() == "fp64"
    Xf = np.clip(X + 0.01, 0, 1)
    with GenotypeSession(Xf) as s:
        s.set_grm("auto")
        s.gblup(idx, Y[idx])
        assert s.grm_used() == "fp64"
        s.set_grm("exact")
        with pytest.raises(gbm.ArgumentError, match="not diploid dosages"):
            s.gblup(idx, Y[idx])


@pytest.mark.parametrize("threads,chunk", [("1", "64"), ("3", "100"), ("16", "64"), ("4", "0")])
def test_host_packed_auto_bit_identical_to_device_checked(dosage_case, gbm_env, threads, chunk):
    """fp64 host X under auto / exact is checked and packed to dosage bytes on the HOST
    (GBM_HOST_PACK=1, the default: worker threads, a ring of pinned slots, each chunk uploaded as it is packed)
    instead of uploaded as fp64 and converted on the device (GBM_HOST_PACK=0). Both give the same bits, against the
    oracle; many small chunks (GBM_PACK_CHUNK) reuse every ring slot; one non-dosage cell in the last locus falls
    back to fp64 both ways (auto) or fails (exact); two shards on one device split the threads."""
    X, Y, ref = dosage_case
    n, p = X.shape
    gbm_env.setenv("GBM_PACK_THREADS", threads)
    if chunk != "0":
        gbm_env.setenv("GBM_PACK_CHUNK", chunk)
    out = {}
    for hp in ("1", "0"):
        gbm_env.setenv("GBM_HOST_PACK", hp)
        info = {}
        out[hp] = gbm.gblup_arrays(X, Y, grm="auto", info=info)
        assert info["grm_used"] == "exact"
        check(out[hp], ref)
    for a, b in zip(out["1"], out["0"]):
        assert np.array_equal(np.asarray(a), np.asarray(b))
    Xb = X.copy()
    Xb[n - 1, p - 1] = 0.25  # not a dosage/2, in the last chunk
    refb = oracle.gblup_fit(Xb, Y, 1.0)
    got = {}
    for hp in ("1", "0"):
        gbm_env.setenv("GBM_HOST_PACK", hp)
        info = {}
        got[hp] = gbm.gblup_arrays(Xb, Y, grm="auto", info=info)
        assert info["grm_used"] == "fp64"
        check(got[hp], refb)
        with pytest.raises(gbm.ArgumentError, match="not diploid dosages"):
            gbm.gblup_arrays(Xb, Y, grm="exact")
    for a, b in zip(got["1"], got["0"]):
        assert np.array_equal(np.asarray(a), np.asarray(b))
    gbm_env.setenv("GBM_HOST_PACK", "1")
    two = gbm.gblup_arrays(X, Y, grm="auto", devices=[0, 0])
    check(two, ref)


@pytest.mark.parametrize("threads", ["16", "3"])
def test_fp64_mode_host_packed_pipeline_bit_identical(gbm_env, threads):
    """grm_mode fp64 on dosage-valued fp64 host X (the C-ABI default): every pipeline chunk is packed to bytes on the
    host (GBM_HOST_PACK=1), uploaded at 1 B per cell and standardised from the bytes, the chunk GRMs summed in the
    fp64 path's order — the same bits as the fp64 upload (GBM_HOST_PACK=0), against the oracle; a non-dosage cell
    in a late chunk falls back to the fp64 upload (same bits again); two shards on one device split the threads."""
    n, p = 777, 20000  # p >= 16 384: the pipelined upload (8 chunks + the halving tail at n <= 8192)
    X = oracle.synth_genotypes(61, n, p)
    Y = oracle.synth_phenotypes(X, 62, ntraits=2)
    ref = oracle.gblup_fit(X, Y, 1.0)
    gbm_env.setenv("GBM_PACK_THREADS", threads)
    got = {}
    for hp in ("1", "0"):
        gbm_env.setenv("GBM_HOST_PACK", hp)
        info = {}
        got[hp] = gbm.gblup_arrays(X, Y, grm="fp64", info=info)
        assert info["grm_used"] == "fp64"
        check(got[hp], ref)
    for a, b in zip(got["1"], got["0"]):
        assert np.array_equal(np.asarray(a), np.asarray(b))
    Xb = X.copy()
    Xb[5, p - 3] = 0.3
    refb = oracle.gblup_fit(Xb, Y, 1.0)
    gotb = {}
    for hp in ("1", "0"):
        gbm_env.setenv("GBM_HOST_PACK", hp)
        gotb[hp] = gbm.gblup_arrays(Xb, Y, grm="fp64")
        check(gotb[hp], refb)
    for a, b in zip(gotb["1"], gotb["0"]):
        assert np.array_equal(np.asarray(a), np.asarray(b))
    gbm_env.setenv("GBM_HOST_PACK", "1")
    two = gbm.gblup_arrays(X, Y, grm="fp64", devices=[0, 0])
    check(two, ref)
