# next_rows.jl — reference-side bindings for the §8(f) rows of libgbm.so: device genotype sessions
# (cross-validation fold farming with a GRM cache), REML λ, the GLMNet-equivalent ridge path and
# the Bayesian ridge (BGLR "BRR") Gibbs sampler. `include("next_rows.jl")` after gblup.jl.
# Julia is absent from the build container, so this file is not executed by the test suite; the
# Python mirror (gbm/session.py, gbm/cv.py, gbm/linear.py, gbm/bayes.py) drives the same C ABI
# with the same argument layout (column-major Float64, Int64 dimensions, 0-based row indices).

# ---- sessions: X resident on one GPU; training-set-keyed GRM cache ------------------------------
mutable struct GenotypeSession
    handle::Ptr{Cvoid}
    n::Int64
    p::Int64
end

"""
    GenotypeSession(X::Matrix{Float64}; device=0)

Upload X (entries x loci-alleles) once to `device`. Replaces the per-fold re-extraction of
`cvmultithread!` (src/cross_validation.jl:159-186): fits on entry subsets gather the training
rows on the device, and their standardised genotypes + GRM are cached per training set.
"""
function GenotypeSession(X::Matrix{Float64}; device::Integer = 0)
    n, p = size(X)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    GC.@preserve X begin
        rc = ccall((:gbm_session_create, LIBGBM), Cint,
                   (Ptr{Float64}, Int64, Int64, Int64, Cint, Ptr{Ptr{Cvoid}}),
                   X, n, p, stride(X, 2), device, h)
    end
    gbm_check(rc, "GenotypeSession")
    s = GenotypeSession(h[], n, p)
    finalizer(s) do s
        s.handle == C_NULL || ccall((:gbm_session_destroy, LIBGBM), Cvoid, (Ptr{Cvoid},), s.handle)
        s.handle = C_NULL
    end
    s
end

# 1-based Julia entry indices -> the ABI's 0-based, strictly increasing rows
zero_based(idx::Vector{Int64}) = issorted(idx) ? idx .- 1 : throw(ArgumentError("entry indices must be increasing"))

"""GBLUP on the rows `idx_training` of the session (phenotypes y, one column per trait)."""
function session_gblup(s::GenotypeSession, idx_training::Vector{Int64}, Y::Matrix{Float64}; λ::Float64 = 1.0)
    idx = zero_based(idx_training)
    m, t = size(Y)
    b_hat = zeros(s.p + 1, t); y_pred = zeros(m, t); mu = zeros(t); q = zeros(Int64, 1)
    GC.@preserve idx Y b_hat y_pred mu q begin
        rc = ccall((:gbm_session_gblup_fit, LIBGBM), Cint,
                   (Ptr{Cvoid}, Ptr{Int64}, Int64, Ptr{Float64}, Int64, Int64, Float64,
                    Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Int64}),
                   s.handle, idx, m, Y, m, t, λ, b_hat, y_pred, mu, q)
    end
    gbm_check(rc, "session_gblup")
    b_hat, y_pred
end

"""`b_hat[1] .+ X[idx, :]*b_hat[2:end]` on the device (reference predict, src/prediction.jl:228)."""
function session_predict(s::GenotypeSession, idx_validation::Vector{Int64}, b_hat::Vector{Float64})
    idx = zero_based(idx_validation)
    out = zeros(length(idx))
    GC.@preserve idx b_hat out begin
        rc = ccall((:gbm_session_predict, LIBGBM), Cint,
                   (Ptr{Cvoid}, Ptr{Int64}, Int64, Ptr{Float64}, Int64, Int64, Ptr{Float64}, Int64),
                   s.handle, idx, length(idx), b_hat, length(b_hat), 1, out, length(idx))
    end
    gbm_check(rc, "session_predict")
    out
end

"""REML λ = σ²_e/σ²_u with the reference's loglikreml objective (src/gwas.jl:450-483)."""
function session_reml(s::GenotypeSession, idx_training::Vector{Int64}, y::Vector{Float64})
    idx = zero_based(idx_training)
    out = zeros(4)
    GC.@preserve idx y out begin
        rc = ccall((:gbm_session_reml, LIBGBM), Cint,
                   (Ptr{Cvoid}, Ptr{Int64}, Int64, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                    Ptr{Float64}),
                   s.handle, idx, length(idx), y, pointer(out, 1), pointer(out, 2), pointer(out, 3), pointer(out, 4))
    end
    gbm_check(rc, "session_reml")
    (λ = out[1], σ²_e = out[2], σ²_u = out[3], objective = out[4])
end

# ---- GLMNet-equivalent ridge path (replaces GLMNet.glmnetcv in ridge, src/linear.jl:193-203) ----
"""
    gpu_glmnetcv_ridge(X, y; nlambda=100, lambda_min_ratio=0.01, nfolds=min(10, n ÷ 3))

Returns a NamedTuple with the fields `ridge` reads from GLMNet's result (`meanloss`, `path.a0`,
`path.betas`, `lambda`): the exact α = 0, standardize = false, intercept solutions on glmnet's λ
sequence and GLMNet.jl's fold scheme, solved on the GPU. Drop-in for the `glmnetcv` call at
src/linear.jl:193-203; the selection loop after it (src/linear.jl:213-221) stays unchanged.
"""
function gpu_glmnetcv_ridge(X::Matrix{Float64}, y::Vector{Float64}; nlambda::Int = 100,
                            lambda_min_ratio::Float64 = 0.01, nfolds::Int = min(10, div(length(y), 3)))
    n, p = size(X)
    s = GenotypeSession(X)
    all = collect(0:(n-1))
    lmax = Ref(0.0)
    GC.@preserve all y begin
        gbm_check(ccall((:gbm_session_ridge_lambda_max, LIBGBM), Cint,
                        (Ptr{Cvoid}, Ptr{Int64}, Int64, Ptr{Float64}, Ptr{Float64}),
                        s.handle, all, n, y, lmax), "ridge_lambda_max")
    end
    λ = lmax[] .* lambda_min_ratio .^ ((0:(nlambda-1)) ./ (nlambda - 1))
    path = zeros(p + 1, nlambda)
    GC.@preserve all y λ path begin
        gbm_check(ccall((:gbm_session_ridge_path, LIBGBM), Cint,
                        (Ptr{Cvoid}, Ptr{Int64}, Int64, Ptr{Float64}, Ptr{Float64}, Int64, Ptr{Float64},
                         Ptr{Int64}, Int64, Ptr{Float64}),
                        s.handle, all, n, y, λ, nlambda, path, C_NULL, 0, C_NULL), "ridge_path")
    end
    q, r = divrem(n, nfolds)
    folds = shuffle!([repeat(1:nfolds, outer = q); 1:r])  # GLMNet.jl's default folds
    loss = zeros(nlambda, nfolds)
    for f = 1:nfolds
        tr = findall(folds .!= f) .- 1; ho = findall(folds .== f) .- 1
        ytr = y[tr .+ 1]
        pf = zeros(p + 1, nlambda); pred = zeros(length(ho), nlambda)
        GC.@preserve tr ho ytr λ pf pred begin
            gbm_check(ccall((:gbm_session_ridge_path, LIBGBM), Cint,
                            (Ptr{Cvoid}, Ptr{Int64}, Int64, Ptr{Float64}, Ptr{Float64}, Int64, Ptr{Float64},
                             Ptr{Int64}, Int64, Ptr{Float64}),
                            s.handle, tr, length(tr), ytr, λ, nlambda, pf, ho, length(ho), pred), "ridge_path")
        end
        loss[:, f] = vec(mean((pred .- y[ho .+ 1]) .^ 2, dims = 1))
    end
    (lambda = λ, meanloss = vec(mean(loss, dims = 2)), path = (a0 = path[1, :], betas = path[2:end, :]))
end

# ---- Bayesian ridge regression (replaces the Rscript/BGLR round trip of bglr(), src/bayes.jl:28-105)
"""
    bglr_brr_gpu(; G, y, n_iter=1_500, n_burnin=500, thin=5, seed=42)::Vector{Float64}

BGLR model "BRR" on the GPU: returns `[posterior mean μ; posterior means b]`, the vector `bglr`
returns for `model="BRR"` (src/bayes.jl:96-104), so `bayesian` uses it unchanged.
"""
function bglr_brr_gpu(; G::Matrix{Float64}, y::Vector{Float64}, n_iter::Int64 = 1_500, n_burnin::Int64 = 500,
                      thin::Int64 = 5, seed::UInt64 = UInt64(42), device::Integer = 0)
    n, p = size(G)
    b_hat = zeros(p + 1)
    GC.@preserve G y b_hat begin
        rc = ccall((:gbm_brr_fit, LIBGBM), Cint,
                   (Ptr{Float64}, Int64, Int64, Int64, Ptr{Float64}, Int64, Int64, Int64, Float64, Float64,
                    UInt64, Cint, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}),
                   G, n, p, stride(G, 2), y, n_iter, n_burnin, thin, 0.5, 5.0, seed, device, b_hat, C_NULL, C_NULL)
    end
    gbm_check(rc, "bglr_brr_gpu")
    msg = unsafe_string(ccall((:gbm_last_error, LIBGBM), Cstring, ()))
    startswith(msg, "warning") && @warn msg  # sweep timed out; re-run on the per-launch path (valid results)
    b_hat
end

# ---- ploidy-aware GRM -----------------------------------------------------------------------
"""
    grmploidyaware_gpu(X::Matrix{Float64}; ploidy=round(Int, 1 / minimum(X[X .!= 0.0])))

Replaces `grmploidyaware(genomes, ploidy=ploidy).genomic_relationship_matrix` at
src/gwas.jl:117-121 (X = the allele frequencies `gwasprep` extracted; the default ploidy is the
caller's own inference, :119). G = k (X − 1fᵀ)(X − 1fᵀ)ᵀ / Σ f(1 − f), f = column means (VanRaden
2008 for ploidy k; GenomicBreedingCore's implementation is un-vendored, so this is the restated
standard form).
"""
function grmploidyaware_gpu(X::Matrix{Float64}; ploidy::Integer = Int(round(1 / minimum(X[X .!= 0.0]))))
    n, p = size(X)
    G = Matrix{Float64}(undef, n, n)
    den = Ref{Float64}(0.0)
    GC.@preserve X G begin
        rc = ccall((:gbm_grm_ploidy_aware, LIBGBM), Cint,
                   (Ptr{Float64}, Int64, Int64, Int64, Cint, Ptr{Int32}, Cint, Ptr{Float64}, Int64, Ptr{Float64}),
                   X, n, p, stride(X, 2), ploidy, C_NULL, 0, G, n, den)
    end
    gbm_check(rc, "grmploidyaware_gpu")
    return G
end
