/*
 * gbm.h — C ABI of the MI355X-native GRM + GBLUP core (libgbm.so).
 *
 * This is the drop-in boundary for GenomicBreedingModels.jl's model-function path
 * (SURVEY.md §8b). A Julia `gblup(; genomes, phenomes, idx_entries, idx_loci_alleles,
 * idx_trait, verbose, λ)::Fit` built exactly like `ridge` (reference src/linear.jl:162-239)
 * calls `gbm_gblup_fit` where `ridge` calls `GLMNet.glmnetcv` (src/linear.jl:193-203);
 * the Julia/ctypes bindings are shown in INTEGRATION.md.
 *
 * Conventions
 *  - All matrices crossing the host entry points are Julia column-major Float64:
 *    X[i, j] lives at X[i + j*ldx] (i = entry/individual, j = locus-allele/SNP).
 *    A SNP column is therefore contiguous, and the device view of X is the row-major
 *    p x n matrix Xt ("locus rows"), whose rows are loaded coalesced along individuals.
 *  - The model is V = G + λI with G = Z Zᵀ / q, Z the column-standardised (ddof = 1)
 *    genotypes over the q non-monomorphic loci (reference src/gwas.jl:112-115,127-130;
 *    V = σ²_u·GRM + σ²_e·I with Z = I at src/gwas.jl:462-471, λ = σ²_e/σ²_u).
 *  - Fixed effect: GLS intercept μ̂ = 1ᵀV⁻¹y / 1ᵀV⁻¹1 (src/gwas.jl:596-597 with X = 1).
 *  - GEBVs / y_pred = μ̂ + G·a with a = V⁻¹(y − 1μ̂).
 *  - b_hat = [b0; b] with b_j = (Zᵀa)_j / (q·s_j) for kept loci (0 for monomorphic ones)
 *    and b0 = μ̂ − Σ_j m_j b_j, so the reference's linear `predict`
 *    (`b_hat[1] .+ X*b_hat[2:end]`, src/prediction.jl:228) reproduces y_pred exactly.
 *  - Return codes: 0 on success, negative GBM_E_* on failure; gbm_last_error() returns a
 *    thread-local message for the last failing call on the calling thread.
 *  - Re-entrant: every call leases its own pooled context (stream + device buffers) per
 *    SNP shard and returns it afterwards; concurrent calls (as `cvmultithread!` makes,
 *    src/cross_validation.jl:159) never share one. Pooled buffers only grow, so repeated calls
 *    of one shape allocate no device memory (gbm_device_allocations); gbm_release_device_cache
 *    frees the idle ones.
 *  - Devices: an explicit `devices` list gives one SNP-column shard per entry (an ordinal may
 *    repeat). With devices == NULL / ndev == 0, each calling thread is given one device,
 *    round-robin over GBM_DEVICES ("0,1,2,..."; re-read per call) or over all visible devices:
 *    the k-th thread to call gets entry k mod len — folds farmed over the GPUs under an
 *    unchanged `cvmultithread!`.
 */
#ifndef GBM_H
#define GBM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GBM_VERSION 212 /* 0.2.1.2: knobs read once (gbm_debug_set), gbm_dev_grm_exact_status */

#define GBM_OK 0
#define GBM_E_ARG (-1)    /* bad argument (ArgumentError on the Julia side, src/prediction.jl:67-127 style) */
#define GBM_E_NOTPD (-2)  /* G + λI not positive definite (non-finite input or λ <= 0) */
#define GBM_E_HIP (-3)    /* HIP runtime error */
#define GBM_E_RCCL (-4)   /* RCCL error */
#define GBM_E_OOM (-5)    /* device allocation failed */
#define GBM_E_NODEV (-6)  /* no usable MI355X device */
#define GBM_E_DATA (-7)   /* data problem: < 2 entries, zero phenotype variance, no polymorphic locus */

/* GRM arithmetic of a fit (the grm_mode argument of the _ex entries and gbm_session_set_grm_mode):
 *   GBM_GRM_FP64   the fp64-MFMA SYRK of the standardised genotypes (the north star's GRM; any X).
 *   GBM_GRM_EXACT  the exact-integer GRM of diploid dosages (int8-MFMA digit GEMMs + int128 centring, one fp64
 *                  rounding): X must hold dosages/2, i.e. 2x exactly 0, 1 or 2 in every cell
 *                  (the allele frequencies extractxyetc hands a diploid gblup, src/prediction.jl:129), int8
 *                  input needs ploidy 2; otherwise GBM_E_ARG. More accurate than fp64 and ~3x faster.
 *   GBM_GRM_AUTO   EXACT when the genotypes are diploid dosages (checked on the device: for fp64 X while it is
 *                  converted to bytes, one chunk of loci first), else FP64.
 *   GBM_GRM_DEFAULT the environment variable GBM_GRM ("fp64" | "exact" | "auto"; read once, gbm_debug_set), else FP64.
 *   GBM_GRM_DROPIN  GBM_GRM when it is set, else AUTO: the default of the drop-in gblup (Julia and Python), so a
 *                   GBM_GRM=fp64 set by a user or CI pins the fp64 SYRK there as everywhere else.
 * The entries without _ex pass GBM_GRM_DEFAULT. */
#define GBM_GRM_DEFAULT (-1)
#define GBM_GRM_FP64 0
#define GBM_GRM_EXACT 1
#define GBM_GRM_AUTO 2
#define GBM_GRM_DROPIN 3

/* Library version (GBM_VERSION) — used by bindings to check the ABI. */
int gbm_version(void);

/* Message for the last failing call on this thread ("" if none). Never NULL. */
const char* gbm_last_error(void);

/* Number of visible HIP devices (0 when none). Returns GBM_OK or GBM_E_HIP. */
int gbm_device_count(int* count);

/* Device allocations (hipMalloc calls) libgbm has made since it was loaded. */
int64_t gbm_device_allocations(void);

/* Free the idle pooled fit contexts of the GBLUP and BRR entries (device buffers, streams and the
 * BRR iteration graphs kept between calls). */
int gbm_release_device_cache(void);

/* --------------------------------------------------------------------------------------
 * Host-buffer entry points (what a Julia `ccall` binds; buffers owned by the caller,
 * no pointer is retained after return).
 * ------------------------------------------------------------------------------------ */

/*
 * GBLUP fit of nrhs traits that share the same entries and loci.
 *   X          n x p column-major allele frequencies (ldx >= n); replaces the matrix that
 *              `extractxyetc(...; add_intercept=false)` returns (src/prediction.jl:129)
 *   Y          n x nrhs column-major phenotypes (ldy >= n), already filtered for missing
 *              values (src/prediction.jl:114-124)
 *   lambda     λ = σ²_e/σ²_u > 0
 *   devices    device ordinals (NULL/ndev = 0: this thread's device, see "Devices" above).
 *              With ndev > 1 SNP columns are sharded into contiguous blocks, one per entry;
 *              the partial GRMs of shards on one device are added there, and summed across
 *              devices with an RCCL all-reduce (communicators cached per device set).
 * Outputs (caller allocated):
 *   b_hat_out  (p+1) x nrhs column-major: [b0; b_1..b_p] per trait (src/linear.jl:218-221 layout)
 *   y_pred_out n x nrhs column-major GEBVs (= fitted values)
 *   mu_out     nrhs GLS intercepts μ̂ (may be NULL)
 *   q_out      number of polymorphic loci used (may be NULL)
 * Replaces: GLMNet.glmnetcv(X, y; alpha=0, ...) + coefficient selection, src/linear.jl:193-221.
 */
int gbm_gblup_fit(const double* X, int64_t n, int64_t p, int64_t ldx,
                  const double* Y, int64_t ldy, int64_t nrhs, double lambda,
                  const int* devices, int ndev,
                  double* b_hat_out, double* y_pred_out, double* mu_out, int64_t* q_out);

/* gbm_gblup_fit with the GRM arithmetic chosen per call (grm_mode: GBM_GRM_*); grm_used_out (may be NULL)
 * receives GBM_GRM_FP64 or GBM_GRM_EXACT, the GRM the fit used. The same for the entries below. */
int gbm_gblup_fit_ex(const double* X, int64_t n, int64_t p, int64_t ldx,
                     const double* Y, int64_t ldy, int64_t nrhs, double lambda,
                     const int* devices, int ndev, int grm_mode,
                     double* b_hat_out, double* y_pred_out, double* mu_out, int64_t* q_out, int* grm_used_out);

/*
 * gbm_gblup_fit with λ chosen per trait by REML — the drop-in `gblup(...; λ = :reml)` (Julia) /
 * `lambda_="reml"` (Python mirror). For each trait column, on the summed GRM of the call (built
 * once): minimise reference loglikreml (src/gwas.jl:450-483 with X = 1, V = σ²_u GRM + σ²_e I) for
 * y standardised as gwasprep does (src/gwas.jl:127-128), over the box σ²_e, σ²_u ∈ [eps, 1]
 * (src/gwas.jl:585; gwasreml's LBFGS at :577-590), σ²_u profiled in closed form per λ = σ²_e/σ²_u and
 * a scan + golden-section search over log λ (the same search as gbm_session_reml); then the GBLUP fit
 * of that trait at its λ (the original, unstandardised y). Outputs as gbm_gblup_fit, plus per trait
 * (nrhs each, any may be NULL): lambda_out, sigma2_e_out, sigma2_u_out. n >= 3.
 */
int gbm_gblup_fit_reml(const double* X, int64_t n, int64_t p, int64_t ldx,
                       const double* Y, int64_t ldy, int64_t nrhs,
                       const int* devices, int ndev,
                       double* b_hat_out, double* y_pred_out, double* mu_out, int64_t* q_out,
                       double* lambda_out, double* sigma2_e_out, double* sigma2_u_out);
int gbm_gblup_fit_reml_ex(const double* X, int64_t n, int64_t p, int64_t ldx,
                          const double* Y, int64_t ldy, int64_t nrhs,
                          const int* devices, int ndev, int grm_mode,
                          double* b_hat_out, double* y_pred_out, double* mu_out, int64_t* q_out,
                          double* lambda_out, double* sigma2_e_out, double* sigma2_u_out, int* grm_used_out);

/*
 * Same as gbm_gblup_fit for int8 dosages: X[i, j] = D[i + j*ldd] / ploidy (exact in fp64).
 * 1 byte per genotype cell over PCIe instead of 8.
 */
int gbm_gblup_fit_dosage_i8(const int8_t* D, int64_t n, int64_t p, int64_t ldd, int ploidy,
                            const double* Y, int64_t ldy, int64_t nrhs, double lambda,
                            const int* devices, int ndev,
                            double* b_hat_out, double* y_pred_out, double* mu_out, int64_t* q_out);
int gbm_gblup_fit_dosage_i8_ex(const int8_t* D, int64_t n, int64_t p, int64_t ldd, int ploidy,
                               const double* Y, int64_t ldy, int64_t nrhs, double lambda,
                               const int* devices, int ndev, int grm_mode,
                               double* b_hat_out, double* y_pred_out, double* mu_out, int64_t* q_out,
                               int* grm_used_out);

/*
 * Same as gbm_gblup_fit on the synthetic genotypes of gbm_dev_synth_genotypes (seed, loci
 * 0..p-1), generated on each device for its SNP-column shard: benchmark-scale
 * fits (config C3: 240 GB of fp64 X) with no host copy of X and no PCIe transfer.
 */
int gbm_gblup_fit_synthetic(uint64_t seed, int64_t n, int64_t p,
                            const double* Y, int64_t ldy, int64_t nrhs, double lambda,
                            const int* devices, int ndev,
                            double* b_hat_out, double* y_pred_out, double* mu_out, int64_t* q_out);
int gbm_gblup_fit_synthetic_ex(uint64_t seed, int64_t n, int64_t p,
                               const double* Y, int64_t ldy, int64_t nrhs, double lambda,
                               const int* devices, int ndev, int grm_mode,
                               double* b_hat_out, double* y_pred_out, double* mu_out, int64_t* q_out,
                               int* grm_used_out);

/*
 * Genomic relationship matrix only: G = Z Zᵀ / q (n x n, column-major == row-major since
 * symmetric, ldg >= n). Replaces GenomicBreedingCore.grmsimple(genomes).genomic_relationship_matrix
 * at src/gwas.jl:124-125 under the north-star formula (the Core implementation is un-vendored).
 */
int gbm_grm(const double* X, int64_t n, int64_t p, int64_t ldx, const int* devices, int ndev,
            double* G_out, int64_t ldg, int64_t* q_out);

/*
 * Ploidy-aware genomic relationship matrix, replacing
 * GenomicBreedingCore.grmploidyaware(genomes, ploidy=ploidy).genomic_relationship_matrix at
 * src/gwas.jl:117-121 (its caller infers ploidy = round(1 / min nonzero X), :119). The Core
 * implementation is un-vendored (parity unpinned); restated as VanRaden (2008) generalised to
 * ploidy k: with f_j = mean_i X[i, j] (allele frequency) and dosages kX,
 *   G = (kX − k1fᵀ)(kX − k1fᵀ)ᵀ / (k Σ_j f_j (1 − f_j)) = k (X − 1fᵀ)(X − 1fᵀ)ᵀ / Σ_j f_j (1 − f_j).
 * Every column is used (monomorphic ones centre to zero). denom_out (may be NULL) = Σ_j f_j (1 − f_j).
 * Same sharding over devices as gbm_grm.
 */
int gbm_grm_ploidy_aware(const double* X, int64_t n, int64_t p, int64_t ldx, int ploidy,
                         const int* devices, int ndev, double* G_out, int64_t ldg, double* denom_out);

/*
 * Column statistics of X: mean, std (ddof = 1, Julia `std`), keep = (std > eps(Float64) and
 * finite), q = Σ keep. Mirrors src/gwas.jl:112-113. Any of mean/sd/keep may be NULL.
 */
int gbm_colstats(const double* X, int64_t n, int64_t p, int64_t ldx, int device,
                 double* mean_out, double* sd_out, uint8_t* keep_out, int64_t* q_out);

/*
 * Linear predictor of `predict` (src/prediction.jl:228): out[i, t] = b_hat[0, t] + Σ_j X[i, j] b_hat[1 + j, t].
 * X n x p column-major (ldx >= n); b_hat (p+1) x nrhs column-major; out n x nrhs column-major.
 */
int gbm_predict(const double* X, int64_t n, int64_t p, int64_t ldx,
                const double* b_hat, int64_t ldb, int64_t nrhs, int device,
                double* out, int64_t ldo);

/* --------------------------------------------------------------------------------------
 * Device-level, stream-ordered entry points (all pointers are device pointers, `stream`
 * is a hipStream_t or NULL for the null stream). Nothing here synchronises the stream.
 * These are the stages the host entry points are built from; the multi-process
 * (one rank per GPU, RCCL all-reduce between grm and solve) path calls them directly.
 *
 * Device layout ("plan geometry", all row-major):
 *   Xt  p x ldx,  ldx >= gbm_dev_npad(n): locus j's n genotypes in Xt[j*ldx + 0..n-1]
 *   G   gbm_dev_gdim(n) x gbm_dev_gdim(n) with ld == gbm_dev_gdim(n): the GRM occupies
 *       rows/cols [0, npad); rows [npad, gdim) are the bordered right-hand sides used by
 *       the fused forward substitution of the Cholesky.
 * ------------------------------------------------------------------------------------ */

/* Padded individual count (multiple of the 128-row tile). */
int64_t gbm_dev_npad(int64_t n);
/* Dimension of the bordered V matrix: npad + 64 (room for 1 + nrhs <= 64 right-hand sides). */
int64_t gbm_dev_gdim(int64_t n);
/* Bytes of device workspace gbm_dev_grm needs for (n, p). */
int64_t gbm_dev_grm_workspace(int64_t n, int64_t p);
/* Bytes of device workspace gbm_dev_gblup_solve needs for (n, nrhs). */
int64_t gbm_dev_solve_workspace(int64_t n, int64_t nrhs);

/* Fill Xt with synthetic genotypes: locus (j0 + j) of a counter-based hash of (seed, i, j0 + j);
 * MAF f ~ U(0.05, 0.5) per locus, dosage ~ Binomial(2, f), X = dosage / 2.
 * Bit-identical to oracle/gbm_oracle.c:gbm_ref_synth_genotype. Zero-fills columns [n, ldx). */
int gbm_dev_synth_genotypes(double* Xt, int64_t ldx, int64_t p, int64_t n, uint64_t seed,
                            int64_t j0, void* stream);

/* The same synthetic genotypes as int8 dosages d = 2X (0, 1, 2), column-major n x p (ldd >= n):
 * locus j0 + j's n dosages at D + j*ldd. 1 byte per cell — the device-resident input of the
 * loci-streamed fit (config C3 on one GPU: 30 GB instead of 240 GB of fp64 X). */
int gbm_dev_synth_dosage_i8(int8_t* D, int64_t ldd, int64_t p, int64_t n, uint64_t seed, int64_t j0,
                            void* stream);

/* Expand int8 dosages (column-major D, n x p, ldd) into Xt (row-major p x ldx) as D/ploidy. */
int gbm_dev_expand_dosage_i8(const int8_t* D, int64_t ldd, int64_t n, int64_t p, int ploidy,
                             double* Xt, int64_t ldx, void* stream);

/* Zt row j <- (x_j − m_j)/s_j for kept loci, 0 for dropped ones and for the padding columns
 * [n, ldz). Zt may be Xt itself (in place, ldz == ldx). Writes mean/sd (p each), keep (p, int32)
 * and atomically adds the kept count into *q_dev (caller zeroes it). Replaces the column std,
 * monomorphic filter and standardisation of reference src/gwas.jl:112-115,127-130. */
int gbm_dev_standardize(const double* Xt, int64_t ldx, int64_t p, int64_t n, double* Zt, int64_t ldz,
                        double* mean, double* sd, int32_t* keep, int64_t* q_dev, void* stream);
/* As gbm_dev_standardize straight from int8 dosage rows (column-major D, n x p, ldd >= n; x = d/ploidy):
 * bit-identical to gbm_dev_expand_dosage_i8 followed by gbm_dev_standardize, out of place into Zt. */
int gbm_dev_standardize_i8(const int8_t* D, int64_t ldd, int64_t p, int64_t n, int ploidy, double* Zt, int64_t ldz,
                           double* mean, double* sd, int32_t* keep, int64_t* q_dev, void* stream);
/* As gbm_dev_standardize over the entry subset idx[0..n) of Xt's columns (gathered in the same
 * pass; out of place): the training-set extraction of reference src/prediction.jl:129 fused
 * with the standardisation. center_only != 0 centres without scaling and keeps every column
 * (sd reported as 1): the X that GLMNet sees with standardize=false (src/linear.jl:193-203). */
int gbm_dev_standardize_gather(const double* Xt, int64_t ldx, int64_t p, const int32_t* idx, int64_t n,
                               double* Zt, int64_t ldz, double* mean, double* sd, int32_t* keep,
                               int64_t* q_dev, int center_only, void* stream);

/* G[0:npad, 0:npad] (upper-triangular 128x128 tiles: rows <= columns) = Σ_j z_j z_jᵀ over
 * the p locus rows of Zt (unscaled: the RCCL all-reduce of multi-GPU shards sums this).
 * Zt and G 16-byte aligned, ldz and ldg even and >= gbm_dev_npad(n).
 * fp64 MFMA SYRK; = gbm_dev_grm_syrk followed by gbm_dev_grm_reduce. Replaces the GRM product
 * of GenomicBreedingCore.grmsimple (called at reference src/gwas.jl:124). */
int gbm_dev_grm(const double* Zt, int64_t ldz, int64_t p, int64_t n, double* G, int64_t ldg,
                void* workspace, int64_t ws_bytes, void* stream);
/* G += Σ_j z_j z_jᵀ over these p locus rows (same tiles and workspace as gbm_dev_grm): the loci-streamed
 * fit adds each chunk of loci into one G. Needs a multi-range plan (gbm_dev_grm_slices(n, p) > 1). */
int gbm_dev_grm_accumulate(const double* Zt, int64_t ldz, int64_t p, int64_t n, double* G, int64_t ldg,
                           void* workspace, int64_t ws_bytes, void* stream);
/* The two launches of gbm_dev_grm, separately (so a caller can time the SYRK kernel alone).
 * The SYRK splits the loci into ranges (gbm_dev_grm_slices of them) and writes one partial tile
 * per range into the workspace, which the reduce sums into G in a fixed order (bit-reproducible
 * run to run); with a single range the SYRK writes G directly and the reduce is a no-op. */
int gbm_dev_grm_syrk(const double* Zt, int64_t ldz, int64_t p, int64_t n, double* G, int64_t ldg,
                     void* workspace, int64_t ws_bytes, void* stream);
int gbm_dev_grm_reduce(int64_t n, int64_t p, double* G, int64_t ldg, const void* workspace, void* stream);
/* The upper 128x128 tiles of G as one contiguous array (packed size in doubles; pack; unpack):
 * half the bytes of G's npad x gdim rows, the form the multi-GPU partial-GRM all-reduce moves. */
int64_t gbm_dev_grm_packed_size(int64_t n);
int gbm_dev_grm_pack(const double* G, int64_t ldg, int64_t n, double* packed, void* stream);
int gbm_dev_grm_unpack(const double* packed, int64_t n, double* G, int64_t ldg, void* stream);
/* Number of loci ranges (split-K slices) the GRM plan uses for (n, p) on the current device. */
int gbm_dev_grm_slices(int64_t n, int64_t p);

/*
 * Solve the GBLUP system on G (as left by gbm_dev_grm, summed over shards):
 *   V = G/q + λI ; LLᵀ = V (blocked fp64 Cholesky, in place) ; μ̂ = 1ᵀV⁻¹y/1ᵀV⁻¹1,
 *   a = V⁻¹(y − 1μ̂), gebv = μ̂ + (y − 1μ̂) − λa  (reference src/gwas.jl:462-472,591-597).
 *   inv_q / q_dev  1/q given on the host, or (q_dev != NULL) read on the device from *q_dev
 *   Y      nrhs x ldy row-major (trait t's n phenotypes contiguous), 1 <= nrhs <= 63
 *   A_out  nrhs x lda row-major: a vectors (lda >= npad; zero in the padding)
 *   gebv   nrhs x lda row-major; mu nrhs; info (device int32): 0 or the 1-based failing pivot.
 *   workspace  >= gbm_dev_solve_workspace(n, nrhs) bytes.
 */
int gbm_dev_gblup_solve(double* G, int64_t ldg, int64_t n, double inv_q, const int64_t* q_dev, double lambda,
                        const double* Y, int64_t ldy, int64_t nrhs,
                        double* A_out, double* gebv, int64_t lda, double* mu, int32_t* info,
                        void* workspace, int64_t ws_bytes, void* stream);

/*
 * The same solve in phases, for a factorisation distributed over ranks (one process or device per
 * rank, each holding the full summed G): gbm_dev_gblup_solve == prepare; for kb = 0 .. npad/64 − 1
 * step gbm_dev_chol_group_size(n, kb): group(kb, rank = 0, nranks = 1); finish.
 * Distributed (nranks > 1, groups of >= 2 panels starting on a 128-row boundary), per group:
 *   [after an earlier distributed group] area_pack(kb, g) → all-gather of gbm_dev_chol_area_doubles
 *                                   per rank → area_unpack; factor_diag(kb): the group's diagonal
 *                                   area (64g x 64g), whose columns other ranks updated;
 *   group_panels(kb, rank, nranks)  the group's panels and row updates on the rank's own 128-column
 *                                   tiles (J ≡ rank mod nranks), the group's diagonal area and the
 *                                   right-hand sides;
 *   strip_pack(kb, g) → all-gather of gbm_dev_chol_strip_doubles per rank → strip_unpack_rows: every
 *                                   rank then holds the group's final rows at every column (and their
 *                                   lower copy, which the back substitution reads);
 *   group_update(kb, rank, nranks)  the trailing update on the rank's own tiles and the right-hand
 *                                   sides — 1/nranks of the O(n³) work per rank (or group_update_tiles
 *                                   over row ranges: the look-ahead, see below).
 * Before switching back to nranks = 1 for the tail, the ranks exchange every remaining row once
 * (strip_pack → all-gather → strip_unpack) and factor its first diagonal block (factor_diag).
 * gbm_dev_chol_group itself takes rank 0 of 1 only (the arguments stay for ABI stability).
 * Bit-identical to gbm_dev_gblup_solve. Replaces the redundant per-rank pinv/Cholesky of V at
 * reference src/gwas.jl:472,595 at multi-GPU scale.
 */
int gbm_dev_chol_prepare(double* G, int64_t ldg, int64_t n, double inv_q, const int64_t* q_dev, double lambda,
                         const double* Y, int64_t ldy, int64_t nrhs, int32_t* info, void* workspace,
                         int64_t ws_bytes, void* stream);
/* gbm_dev_chol_prepare for rank `rank` of a distributed factorisation (nranks > 1): V only on the columns
 * the rank reads before an exchange overwrites them (its own 128-column tiles, the first panel group's
 * area, the right-hand sides); nranks = 1 is gbm_dev_chol_prepare. */
int gbm_dev_chol_prepare_cols(double* G, int64_t ldg, int64_t n, double inv_q, const int64_t* q_dev, double lambda,
                              const double* Y, int64_t ldy, int64_t nrhs, int rank, int nranks, int32_t* info,
                              void* workspace, int64_t ws_bytes, void* stream);
/* Panels in the group that starts at 64-row block kb (0 past the end). At the dataflow tail (at most
 * GBM_CHOL_TAIL_FLOW rows left, default 8192 when npad > 12 288; never kb = 0) every remaining panel:
 * gbm_dev_chol_group then factors the rest in one launch, and group_panels / group_update refuse it. */
int64_t gbm_dev_chol_group_size(int64_t n, int64_t kb);
int gbm_dev_chol_group(double* G, int64_t ldg, int64_t n, int64_t kb, int rank, int nranks, int32_t* info,
                       void* workspace, int64_t ws_bytes, void* stream);
int gbm_dev_chol_group_panels(double* G, int64_t ldg, int64_t n, int64_t kb, int rank, int nranks, int32_t* info,
                              void* workspace, int64_t ws_bytes, void* stream);
int gbm_dev_chol_group_update(double* G, int64_t ldg, int64_t n, int64_t kb, int rank, int nranks, int32_t* info,
                              void* workspace, int64_t ws_bytes, void* stream);
/* group_update restricted to the rank's tiles with columns in [col_lo, col_hi) (col_lo on a 128-column
 * tile; the right-hand sides when col_hi >= gdim(n)); nranks >= 2. Two calls covering [64 (kb + g),
 * gdim) equal one group_update: the first (the next group's area) lets the area exchange run beside
 * the second. */
int gbm_dev_chol_group_update_cols(double* G, int64_t ldg, int64_t n, int64_t kb, int rank, int nranks,
                                   int64_t col_lo, int64_t col_hi, int32_t* info, void* workspace, int64_t ws_bytes,
                                   void* stream);
/* group_update_cols further restricted to the rows [row_lo, row_hi) (row_lo on a 128-row tile): the
 * look-ahead updates the next group's rows first, so that group's panels (group_panels) and row exchange
 * run beside the rest of the update (rows from the end of the next group on). */
int gbm_dev_chol_group_update_tiles(double* G, int64_t ldg, int64_t n, int64_t kb, int rank, int nranks,
                                    int64_t row_lo, int64_t row_hi, int64_t col_lo, int64_t col_hi, int32_t* info,
                                    void* workspace, int64_t ws_bytes, void* stream);
int gbm_dev_chol_factor_diag(double* G, int64_t ldg, int64_t n, int64_t kb, int32_t* info, void* workspace,
                             int64_t ws_bytes, void* stream);
/* Doubles per rank of the strip of rows [64 kb, 64 (kb + rows64)) over the tiles from column 64 kb. */
int64_t gbm_dev_chol_strip_doubles(int64_t n, int64_t kb, int64_t rows64, int nranks);
int gbm_dev_chol_strip_pack(const double* G, int64_t ldg, int64_t n, int64_t kb, int64_t rows64, int rank,
                            int nranks, double* buf, void* stream);
/* gathered: nranks consecutive packs (rank order), e.g. the output of an all-gather. */
int gbm_dev_chol_strip_unpack(double* G, int64_t ldg, int64_t n, int64_t kb, int64_t rows64, int nranks,
                              const double* gathered, void* stream);
/* The same over the square [64 kb, 64 (kb + rows64)) only (rows64 even): a group's diagonal area. */
int64_t gbm_dev_chol_area_doubles(int64_t n, int64_t kb, int64_t rows64, int nranks);
int gbm_dev_chol_area_pack(const double* G, int64_t ldg, int64_t n, int64_t kb, int64_t rows64, int rank,
                           int nranks, double* buf, void* stream);
int gbm_dev_chol_area_unpack(double* G, int64_t ldg, int64_t n, int64_t kb, int64_t rows64, int nranks,
                             const double* gathered, void* stream);
/* The transposed lower copy (read only by gbm_dev_chol_finish) of the rows [64 kb, 64 (kb + rows64)) for the
 * chunks other ranks solved. A driver may defer it to a stream of its own (the rows are final; nothing before
 * finish reads or writes those entries). */
int gbm_dev_chol_lower_copy(double* G, int64_t ldg, int64_t n, int64_t kb, int64_t rows64, int rank, int nranks,
                            void* stream);
/* strip_unpack of final factor rows (after group_panels) plus their lower copy for the columns this
 * rank did not compute (= strip_unpack + lower_copy). */
int gbm_dev_chol_strip_unpack_rows(double* G, int64_t ldg, int64_t n, int64_t kb, int64_t rows64, int rank,
                                   int nranks, const double* gathered, void* stream);
int gbm_dev_chol_finish(double* G, int64_t ldg, int64_t n, const double* Y, int64_t ldy, int64_t nrhs,
                        double lambda, double* A_out, double* gebv, int64_t lda, double* mu, int32_t* info,
                        void* workspace, int64_t ws_bytes, void* stream);

/* REML ingredients of a finished gbm_dev_gblup_solve (same G, workspace, n, nrhs), into device
 * memory: terms[0] = logdet(G/q + λI), terms[1] = 1ᵀV⁻¹1, terms[2+2t] = 1ᵀV⁻¹y_t,
 * terms[3+2t] = y_tᵀV⁻¹y_t — everything reference loglikreml (src/gwas.jl:450-483) needs with
 * X = 1, read off the bordered factorisation. */
int gbm_dev_gblup_terms(const double* G, int64_t ldg, int64_t n, int64_t nrhs, const void* workspace,
                        double* terms, void* stream);

/*
 * Marker effects on the standardised locus rows: B[t, j] = (Zt_j · a_t)/(q·sd_j) for kept
 * loci, 0 otherwise (B nrhs x ldb row-major), and msum[t] = Σ_j mean_j B[t, j] over this
 * shard (so that b0 = μ̂ − Σ_shards msum). q from inv_q or, if q_dev != NULL, from *q_dev.
 */
int gbm_dev_marker_effects(const double* Zt, int64_t ldz, int64_t p, int64_t n,
                           const double* A, int64_t lda, int64_t nrhs, double inv_q, const int64_t* q_dev,
                           const double* mean, const double* sd, const int32_t* keep,
                           double* B, int64_t ldb, double* msum, void* stream);

/* Bytes of device workspace gbm_dev_grm_exact_i8 needs for (n, p): the individual-major operand copies
 * (2 x npad x p bytes), the per-locus digits and the 128-bit centring terms. */
int64_t gbm_dev_grm_exact_workspace(int64_t n, int64_t p);
/* The GRM of diploid dosages (column-major D, n x p, ldd >= n, d in {0, 1, 2}, x = d/2) computed EXACTLY up to
 * the fp64 rounding of each locus weight 1/var_j: G = Σ_j w_j (d_j − t_j/n)(d_j − t_j/n)ᵀ, the GRM of the
 * standardised genotypes (reference src/gwas.jl:112-126 before the 1/q), as int8 MFMA GEMMs over the base-128
 * digits of the fixed-point weights with 128-bit centring. Also writes what
 * gbm_dev_standardize_i8 writes except Z: mean, sd, keep (per locus) and adds the kept count to *q_dev.
 * accum != 0: G += this GRM. *slices_out (optional): the digit count S (8-10) the weights needed.
 * Upper tiles of G are written (ldg >= gbm_dev_npad(n)); one host synchronisation per call (sizes S).
 * GBM_E_ARG on a dosage outside {0, 1, 2} or ploidy != 2. */
int gbm_dev_grm_exact_i8(const int8_t* D, int64_t ldd, int64_t p, int64_t n, int ploidy, double* G, int64_t ldg,
                         double* mean, double* sd, int32_t* keep, int64_t* q_dev, int accum, void* workspace,
                         int64_t ws_bytes, int32_t* slices_out, void* stream);
/* The status a gbm_dev_grm_exact_i8 launch left in its workspace (same n, p, workspace; synchronises the
 * stream): GBM_E_HIP when a locus weight did not fit its S base-128 digits (G invalid; xg_choose's bound rules it
 * out, this makes a violation loud), GBM_E_ARG for a dosage outside {0, 1, 2}, else GBM_OK. The C-ABI fits and
 * sessions call it after every exact GRM. */
int gbm_dev_grm_exact_status(const void* workspace, int64_t n, int64_t p, void* stream);

/* gbm_dev_marker_effects on int8 dosage rows (column-major D, n x p, ldd >= n, x = d/ploidy) instead of the
 * standardised fp64 rows: z = (x − mean_j)/sd_j is rebuilt in registers exactly as gbm_dev_standardize_i8
 * wrote it, so B and msum are bit-identical, at 1 byte read per cell (the loci-streamed fit's back-solve,
 * which keeps no fp64 Z). lda >= gbm_dev_npad(n), even. */
int gbm_dev_marker_effects_i8(const int8_t* D, int64_t ldd, int64_t p, int64_t n, int ploidy,
                              const double* A, int64_t lda, int64_t nrhs, double inv_q, const int64_t* q_dev,
                              const double* mean, const double* sd, const int32_t* keep,
                              double* B, int64_t ldb, double* msum, void* stream);

/*
 * ---- Device-resident genotype sessions: cross-validation fold farming and REML λ -----------
 * A session holds X (n x p, uploaded once) on one device and fits GBLUP on entry subsets; the
 * standardised training genotypes and their GRM are cached per training set, so further traits,
 * λ values and REML evaluations on the same set skip the SYRK. Replaces the per-fold model calls
 * of reference cvmultithread! (src/cross_validation.jl:151-207); use one session per device and
 * one host thread per session. Entry indices are 0-based rows of X, strictly increasing.
 */
typedef struct gbm_session gbm_session;
int gbm_session_create(const double* X, int64_t n, int64_t p, int64_t ldx, int device, gbm_session** out);
int gbm_session_create_dosage_i8(const int8_t* D, int64_t n, int64_t p, int64_t ldd, int ploidy, int device,
                                 gbm_session** out);
/* A session over the synthetic genotypes of gbm_dev_synth_genotypes (seed, loci 0..p-1), generated
 * on the device: benchmark-scale sessions (configs C4/C5) without a host copy of X. */
int gbm_session_create_synthetic(uint64_t seed, int64_t n, int64_t p, int device, gbm_session** out);
void gbm_session_destroy(gbm_session* s);
/* GRM arithmetic of the session's training GRMs (GBM_GRM_*; default GBM_GRM_DEFAULT = the GBM_GRM variable):
 * exact / auto build them with the exact-integer kernels when the genotypes are diploid dosages/2 (checked once
 * on the device). The training-set cache is keyed by the GRM used as well. */
int gbm_session_set_grm_mode(gbm_session* s, int grm_mode);
/* The GRM the cached training set was built with: GBM_GRM_FP64, GBM_GRM_EXACT, or -1 before the first fit. */
int gbm_session_grm_used(gbm_session* s, int* grm_used);
/* gbm_gblup_fit on the rows idx[0..n_train) of the session's X; Y holds the training phenotypes
 * (n_train x nrhs, column-major). */
int gbm_session_gblup_fit(gbm_session* s, const int64_t* idx, int64_t n_train, const double* Y, int64_t ldy,
                          int64_t nrhs, double lambda, double* b_hat_out, double* y_pred_out, double* mu_out,
                          int64_t* q_out);
/* out[t*ldo + i] = b_hat[t*ldb] + X[idx[i], :] · b_hat[t*ldb + 1 : t*ldb + 1 + p] on the device
 * (reference predict, src/prediction.jl:228). */
int gbm_session_predict(gbm_session* s, const int64_t* idx, int64_t n_val, const double* b_hat, int64_t ldb,
                        int64_t nrhs, double* out, int64_t ldo);
/* Reference loglikreml (src/gwas.jl:450-483) with X = 1 (intercept) and GRM = ZZᵀ/q of the
 * training rows: out[k] = 0.5 logdet V + yᵀPy + logdet(XᵀV⁻¹X), V = σ²_u[k] GRM + σ²_e[k] I, for
 * y as given. One Cholesky per (σ²_e, σ²_u) pair. */
int gbm_session_reml_objective(gbm_session* s, const int64_t* idx, int64_t n_train, const double* y,
                               const double* sigma2_e, const double* sigma2_u, int64_t m, double* out);
/* REML choice of λ = σ²_e/σ²_u: minimises that objective for y standardised as gwasprep does
 * (src/gwas.jl:127-128) over the reference's box σ²_e, σ²_u ∈ [eps, 1] (src/gwas.jl:585), with
 * σ²_u profiled in closed form per λ and a scan + golden-section search over log λ. */
int gbm_session_reml(gbm_session* s, const int64_t* idx, int64_t n_train, const double* y, double* lambda_out,
                     double* sigma2_e_out, double* sigma2_u_out, double* objective_out);
/* Ridge path of reference ridge (GLMNet alpha = 0, standardize = false, intercept;
 * src/linear.jl:193-203) on the rows idx[0..n_train): for each lambdas[k] (glmnet scale, objective
 * (1/2n)‖y − a0 − Xb‖² + (λ/2)‖b‖²) the exact minimiser, b_path_out[k*(p+1)] = a0 and
 * b_path_out[k*(p+1) + 1 + j] = b_j; optionally pred_out[k*n_eval + i] = a0 + X[idx_eval[i], :] b. */
int gbm_session_ridge_path(gbm_session* s, const int64_t* idx, int64_t n_train, const double* y,
                           const double* lambdas, int64_t nl, double* b_path_out, const int64_t* idx_eval,
                           int64_t n_eval, double* pred_out);
/* glmnet's largest λ for alpha = 0 (alpha floored at 1e-3): max_j |x_cjᵀ(y − ȳ)| / n / 1e-3. */
int gbm_session_ridge_lambda_max(gbm_session* s, const int64_t* idx, int64_t n_train, const double* y,
                                 double* lambda_max);
/* GRM builds and cache hits so far. */
int gbm_session_stats(gbm_session* s, int64_t* grm_builds, int64_t* grm_hits);

/*
 * ---- Bayesian ridge regression (BGLR model "BRR") by Gibbs sampling -------------------------
 * Replaces the Rscript/BGLR call of reference bglr()/bayesian() (src/bayes.jl:28-105,158-224)
 * for bglr_model = "BRR": BGLR's single-site sampler (intercept, markers in order with residual
 * updates, σ²_b and σ²_e scaled-inverse-χ² draws; priors df0, R2 as BGLR's defaults 5 and 0.5),
 * n_iter iterations, running posterior means every `thin` iterations after n_burnin.
 * b_hat_out (p+1) = [posterior mean of μ; posterior means of b]; y_pred_out (n, optional) =
 * b0 + X b; var_out (2, optional) = posterior means of [σ²_e, σ²_b]. X column-major n x p.
 * Counter-based random numbers from `seed` (no R RNG stream: results are reproducible but the
 * chain is not BGLR's sample path).
 * Schedule: one persistent super-block sweep launch per iteration when its workgroups fit one per CU
 * (byte-exact genotypes, n <= 48 x CUs), else one launch per marker block. If the sweep's
 * inter-workgroup hand-offs time out (its workgroups could not all be resident, e.g. another process
 * fills the device) the fit is re-run from the start on the per-launch path: the call still returns
 * GBM_OK (the results are valid) and gbm_last_error() then holds a message starting "warning:" (it
 * is "" after any other successful call of this function).
 */
int gbm_brr_fit(const double* X, int64_t n, int64_t p, int64_t ldx, const double* y, int64_t n_iter,
                int64_t n_burnin, int64_t thin, double r2, double df0, uint64_t seed, int device,
                double* b_hat_out, double* y_pred_out, double* var_out);

/* --------------------------------------------------------------------------------------
 * Diagnostics (tests and timing tools; no reference counterpart).
 * ------------------------------------------------------------------------------------ */
/* Which schedule the last completed gbm_brr_fit ran (*last_path: 0 one launch per block, 4 the
 * super-block sweep with two super-blocks of slack for the partial dots; 1-3 were earlier sweeps, no
 * longer built) and how many fits so far fell back to the per-launch schedule after a sweep
 * hand-off timed out (*fallbacks). */
int gbm_debug_brr_stats(int* last_path, int64_t* fallbacks);
/* Chunk shape of the last super-block sweep: C workgroups, the first O own R rows of every
 * super-block and take Ko individuals each, the others Kn. */
int gbm_debug_brr_shape(int* C, int* O, int* R, int* Ko, int* Kn);
/* Allocations that ran out of device memory and were retried after freeing the idle pooled contexts
 * (GBLUP and BRR) of their device, and how many contexts those retries freed. */
int gbm_debug_oom_retries(int64_t* retries, int64_t* contexts_freed);
/* With GBM_BRR_TRACE=1 set for a fit: copies up to cap int64 timestamps (100 MHz) of the last
 * super-block sweep into host; returns the count, 0 when no trace was taken, -1 on a HIP error. */
int64_t gbm_debug_brr_trace(int64_t* host, int64_t cap);
/* With GBM_CHOL_FLOW_TRACE=1 set for a solve: copies up to cap records of 24 int64 (tile, workgroup,
 * 100 MHz timestamps) of the last dataflow factorisation into host; returns the record count. */
int64_t gbm_debug_chol_flow_trace(int64_t* host, int64_t cap);
/* The dataflow factorisation's worker dequeue order for nbc 64-tiles per side (host only, no device work; the
 * variant GBM_CHOL_FLOW_ORDER selects): returns 0 when every task follows the tasks it waits for (so the launch
 * completes with ONE worker), else the first failing position + 1 (−1 for a bad nbc); copies the entries
 * (i << 16) | j, with bit 15 set for a task that covers the tiles (i, j) and (i, j + 1), to order_out when cap
 * allows (gbm_debug_chol_flow_order_size entries; nbc (nbc + 1)/2 − 1 tiles in all). */
int64_t gbm_debug_chol_flow_order(int nbc, int32_t* order_out, int64_t cap);
int64_t gbm_debug_chol_flow_order_size(int nbc);
/* The same check of a caller's order (m entries). */
int64_t gbm_debug_chol_flow_order_check(int nbc, const int32_t* order, int64_t m);
/* Successful RCCL collectives libgbm has issued (partial-GRM all-reduces; Cholesky strip all-gathers). With
 * GBM_FORCE_RCCL=1 set for a call, a fit with one device leader still runs them on a 1-rank communicator
 * (the all-gathers from n >= GBM_DIST_SOLVE_MIN_N), bit-identical to the call without: the RCCL path on a
 * one-GPU box. */
int gbm_debug_rccl_calls(int64_t* allreduce, int64_t* allgather);
/* The exact GRM's digit count S and scale exponent F for kept-locus weights in [wmin, wmax] (host only, no
 * device work; returns 1 when every weight is exact on the 2^-F grid, 0 when the smallest are rounded). */
int gbm_debug_xg_choose(double wmin, double wmax, int* slices_out, int* shift_out);
/* Sets (value != NULL) or clears (NULL) a GBM_* tuning/test knob. libgbm reads the environment's GBM_*
 * variables ONCE, at its first knob lookup, and never calls getenv on a fit path afterwards (no race with a
 * setenv in another thread under Threads.@threads); later changes go through this entry only. Thread-safe.
 * GBM_E_ARG unless name starts with "GBM_". */
int gbm_debug_set(const char* name, const char* value);

#ifdef __cplusplus
}
#endif

#endif /* GBM_H */
