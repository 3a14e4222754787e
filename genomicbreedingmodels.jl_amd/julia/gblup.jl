# gblup.jl — the reference-side binding a GenomicBreedingModels.jl maintainer adds to call
# libgbm.so (MI355X GRM + GBLUP core). Drop into src/ next to linear.jl, `include("gblup.jl")`
# after linear.jl (src/GenomicBreedingModels.jl:25-33), export `gblup` next to `ridge`
# (src/GenomicBreedingModels.jl:46) and add "gblup" to `linear_models` in predict
# (src/prediction.jl:225). Julia is not available in the build container, so this file is not
# executed by the test suite; the Python mirror (gbm/linear.py) exercises the same C ABI with
# the same argument layout (column-major Float64, Int64 dimensions).

const LIBGBM = get(ENV, "GBM_LIBRARY", joinpath(@__DIR__, "..", "gbm", "libgbm.so"))

function gbm_last_error()::String
    unsafe_string(ccall((:gbm_last_error, LIBGBM), Cstring, ()))
end

# GRM arithmetic (include/gbm.h GBM_GRM_*): :auto = exact int8-MFMA GRM when the allele frequencies are
# diploid dosages/2 (2x ∈ {0, 1, 2} in every cell, checked on the device), else the fp64-MFMA SYRK
# :dropin (gblup's default) = the GBM_GRM variable when it is set, else :auto
const GBM_GRM_MODES = Dict(:default => Cint(-1), :fp64 => Cint(0), :exact => Cint(1), :auto => Cint(2),
                           :dropin => Cint(3))

function gbm_grm_mode(grm::Symbol)::Cint
    haskey(GBM_GRM_MODES, grm) || throw(ArgumentError("grm must be :dropin, :auto, :exact, :fp64 or :default, got :$grm"))
    GBM_GRM_MODES[grm]
end

function gbm_check(rc::Cint, what::String)
    rc == 0 && return nothing
    msg = what * ": " * gbm_last_error()
    rc == -1 ? throw(ArgumentError(msg)) : throw(ErrorException(msg))
end

"""
    gblup(; genomes, phenomes, idx_entries=nothing, idx_loci_alleles=nothing, idx_trait=1,
          verbose=false, λ=1.0, devices=Int32[], model_label="gblup", grm=:dropin)::Fit

GBLUP / RR-BLUP on V = G + λI with G = ZZᵀ/q, fitted on MI355X GPUs through libgbm.so.
Same keywords and Fit assembly as `ridge` (src/linear.jl:162-239), so it runs unchanged under
`cvbulk`/`cvmultithread!` (src/cross_validation.jl:170-177) and `predict`.
`λ = :reml` chooses λ = σ²_e/σ²_u by REML on the fit's own GRM first (gbm_gblup_fit_reml: the
reference's loglikreml objective, src/gwas.jl:450-483, over gwasreml's box, :577-590); a partial
of `gblup` with `λ = :reml` (e.g. `gblup_reml(; kw...) = gblup(; kw..., λ = :reml)`) then goes into
`cvbulk(models = [...])` unchanged.
`grm = :auto` computes the GRM exactly on the int8 matrix cores when the allele frequencies
are diploid dosages/2 (the usual `Genomes` of a diploid population; ≈3× faster at n = 5 000 and exact up to
each locus weight's fp64 rounding), else with the fp64-MFMA SYRK; `:fp64` / `:exact` force one. The default
`grm = :dropin` is `:auto` unless the environment sets GBM_GRM (fp64 | exact | auto), which then decides.
"""
function gblup(;
    genomes::Genomes,
    phenomes::Phenomes,
    idx_entries::Union{Nothing,Vector{Int64}} = nothing,
    idx_loci_alleles::Union{Nothing,Vector{Int64}} = nothing,
    idx_trait::Int64 = 1,
    verbose::Bool = false,
    λ::Union{Float64,Symbol} = 1.0,
    devices::Vector{Int32} = Int32[],
    model_label::String = "gblup",
    grm::Symbol = :dropin,
)::Fit
    X, y, entries, populations, loci_alleles = extractxyetc(
        genomes,
        phenomes,
        idx_entries = idx_entries,
        idx_loci_alleles = idx_loci_alleles,
        idx_trait = idx_trait,
        add_intercept = false,
    )
    n, p = size(X)
    fit::Fit = Fit(n = n, l = p)
    fit.model = model_label
    fit.b_hat_labels = vcat(["intercept"], loci_alleles)
    fit.trait = phenomes.traits[idx_trait]
    fit.entries = entries
    fit.populations = populations
    fit.y_true = y
    b_hat = zeros(p + 1)
    y_pred = zeros(n)
    mu = zeros(1)
    q = zeros(Int64, 1)
    λ_used = zeros(1)
    σ2 = zeros(2)
    grm_used = Cint[-1]
    mode = gbm_grm_mode(grm)
    devs = isempty(devices) ? C_NULL : pointer(devices)
    GC.@preserve X y b_hat y_pred mu q devices λ_used σ2 grm_used begin
        if λ isa Symbol
            λ === :reml || throw(ArgumentError("λ must be a Float64 or :reml, got :$λ"))
            rc = ccall(
                (:gbm_gblup_fit_reml_ex, LIBGBM),
                Cint,
                (Ptr{Float64}, Int64, Int64, Int64, Ptr{Float64}, Int64, Int64, Ptr{Int32}, Cint, Cint,
                 Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Int64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                 Ptr{Cint}),
                X, n, p, stride(X, 2), y, n, 1, devs, length(devices), mode,
                b_hat, y_pred, mu, q, λ_used, pointer(σ2, 1), pointer(σ2, 2), grm_used,
            )
            gbm_check(rc, "gblup (REML)")
        else
            rc = ccall(
                (:gbm_gblup_fit_ex, LIBGBM),
                Cint,
                (Ptr{Float64}, Int64, Int64, Int64, Ptr{Float64}, Int64, Int64, Float64,
                 Ptr{Int32}, Cint, Cint, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Int64}, Ptr{Cint}),
                X, n, p, stride(X, 2), y, n, 1, λ,
                devs, length(devices), mode,
                b_hat, y_pred, mu, q, grm_used,
            )
            gbm_check(rc, "gblup")
            λ_used[1] = λ
        end
    end
    fit.b_hat = b_hat
    fit.y_pred = y_pred
    fit.metrics = metrics(y, y_pred)
    if verbose
        println("gblup: n=$n p=$p q=$(q[1]) μ̂=$(mu[1]) λ=$(λ_used[1]) grm=$(grm_used[1] == 1 ? "exact" : "fp64")" *
                (λ isa Symbol ? " (REML: σ²_e=$(σ2[1]), σ²_u=$(σ2[2]))" : ""))
        println(fit.metrics)
    end
    if !checkdims(fit)
        throw(ErrorException("Error fitting " * fit.model * "."))
    end
    fit
end
