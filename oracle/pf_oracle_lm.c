/*
 * pf_oracle_lm.c -- CPU restatement of the reference's registration SOLVER: Ceres Solver 1.13's
 * trust-region Levenberg-Marquardt with DENSE_SCHUR and default options, as SolveDepthToDepth
 * calls it (Depth.cpp:1270-1274 vars = (1,1,1,1); :1374-1375 one AutoDiffCostFunction
 * <FunctorDepth2Depth3,1,1,1,1,1> per sample; :1391-1404 AddResidualBlock(a,b,c,d) + Solve with
 * linear_solver_type = DENSE_SCHUR).
 *
 * TEST INFRASTRUCTURE ONLY (see pf_oracle.h).  Ceres is a third-party dependency vendored in the
 * reference (ceres-solver/, VERSION 1.13.0, commit 19333b0f); it is built with CMake and is
 * therefore not buildable here, so its published algorithm is restated from its sources:
 *
 *  - options: include/ceres/solver.h:62-128 (max_num_iterations 50, initial radius 1e4, max
 *    radius 1e16, min radius 1e-32, min_relative_decrease 1e-3, min/max LM diagonal 1e-6/1e32,
 *    max 5 consecutive invalid steps, function_tolerance 1e-6, gradient_tolerance 1e-10,
 *    parameter_tolerance 1e-8, jacobi_scaling on, monotonic steps, no inner iterations);
 *  - the loop: internal/ceres/trust_region_minimizer.cc:66-119 (Minimize), :177-279 (iteration
 *    zero, Jacobi column scaling 1/(1+sqrt(|col|^2)) fixed at iteration 0, gradient max norm as
 *    |x - (x - g)|_inf), :291-335 (termination checks after every iteration), :355-424 (model
 *    cost change -(J s).(r + J s / 2), valid iff > 0), :429-462 (invalid steps), :667-705
 *    (parameter tolerance with x_norm = -1 until the first accepted step; function tolerance
 *    |dcost| <= 1e-6 cost -- both return WITHOUT accepting the candidate), :736-786 (accept iff
 *    relative decrease > 1e-3; the best accepted point is the result, :291-300);
 *  - the step quality: trust_region_step_evaluator.cc:51-104 (monotonic: the plain ratio);
 *  - the LM strategy: levenberg_marquardt_strategy.cc:65-164 (diagonal = clamped squared column
 *    norms of the scaled Jacobian, reused after a rejection; D = sqrt(diag / radius); solve
 *    J y = r, step = -y; accept: radius /= max(1/3, 1 - (2 rho - 1)^3), capped; reject: radius
 *    /= decrease_factor, decrease_factor *= 2);
 *  - DENSE_SCHUR for this problem: parameter_block_ordering.cc:50-79 + graph_algorithms.h:173-
 *    226 make `a` the one eliminated block (every residual touches all four blocks, so the
 *    stable independent set is the first block), f-blocks (b, c, d);
 *    schur_eliminator_impl.h:176-298 (Eliminate: S = D_f^2 + sum F'F - (E'F)' (E'E + D_e^2)^-1
 *    (E'F), rhs = sum F'(r - E (E'E)^-1 E'r), with (E'E)^-1 from a 1x1 Cholesky), the 3x3
 *    reduced system by Eigen's LLT (schur_complement_solver.cc:197-213), back substitution
 *    schur_eliminator_impl.h:303-366.
 *
 * Residual of sample i (FunctorDepth2Depth3, Depth.cpp:1124-1130, Weight = 1, evaluated in
 * double): r = ((X3 a + X2 b) + X c + d) - Y with X2 = x*x, X3 = x*x*x; Jacobian row (X3, X2, X,
 * 1); cost = sum 0.5 r^2 in residual order (ResidualBlock::Evaluate + ProgramEvaluator).
 *
 * Fidelity: the control flow (every branch and constant above) is Ceres's; the linear algebra
 * follows Ceres's/Eigen's operation order for these block sizes but is not guaranteed to
 * reproduce Eigen's bits (its SIMD reduction order), so an LM run here can differ from Ceres
 * only where a termination test lands within rounding of its threshold.
 */
#include "pf_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define LM_MAX_ITER 50
#define LM_INIT_RADIUS 1e4
#define LM_MAX_RADIUS 1e16
#define LM_MIN_RADIUS 1e-32
#define LM_MIN_REL_DECREASE 1e-3
#define LM_MIN_DIAG 1e-6
#define LM_MAX_DIAG 1e32
#define LM_MAX_INVALID 5
#define LM_FUNC_TOL 1e-6
#define LM_GRAD_TOL 1e-10
#define LM_PARAM_TOL 1e-8

typedef struct {
    int n;
    const double *x, *y;
    double* J;  /* n x 4, row-major, scaled in place after each evaluation */
} lm_problem;

/* cost (and optionally residuals, unscaled Jacobian, gradient) at parameters p */
static double lm_evaluate(const lm_problem* P, const double p[4], double* r, double* J, double g[4])
{
    double cost = 0.0;
    if (g) g[0] = g[1] = g[2] = g[3] = 0.0;
    for (int i = 0; i < P->n; i++) {
        const double X = P->x[i], X2 = X * X, X3 = X * X * X, Y = P->y[i];
        const double ri = 1.0 * ((((X3 * p[0] + X2 * p[1]) + X * p[2]) + p[3]) - Y);
        cost = cost + 0.5 * (ri * ri);
        if (r) r[i] = ri;
        if (J) {
            double* row = J + 4 * (size_t)i;
            row[0] = X3; row[1] = X2; row[2] = X; row[3] = 1.0;
        }
        if (g) {
            g[0] = g[0] + X3 * ri;
            g[1] = g[1] + X2 * ri;
            g[2] = g[2] + X * ri;
            g[3] = g[3] + 1.0 * ri;
        }
    }
    return cost;
}

static void col_sqnorm(const double* J, int n, double out[4])
{
    out[0] = out[1] = out[2] = out[3] = 0.0;
    for (int i = 0; i < n; i++)
        for (int k = 0; k < 4; k++) out[k] = out[k] + J[4 * (size_t)i + k] * J[4 * (size_t)i + k];
}

/* 1x1 "InvertPSDMatrix" with the full-rank flag: Eigen LLT of [v], solved against 1 */
static double inv_psd1(double v)
{
    const double l = sqrt(v);
    return (1.0 / l) / l;
}

/* Eigen LLT<Upper> of the 3x3 reduced system and its solve; returns -1 if not positive definite */
static int llt3_solve(double S[3][3], const double rhs[3], double z[3])
{
    double L[3][3] = {{0}};
    for (int k = 0; k < 3; k++) {
        double x = S[k][k];
        if (k > 0) {
            double sq = 0.0;
            for (int i = 0; i < k; i++) sq = sq + L[k][i] * L[k][i];
            x = x - sq;
        }
        if (!(x > 0.0)) return -1;
        L[k][k] = x = sqrt(x);
        for (int j = k + 1; j < 3; j++) {
            double a = S[k][j];  /* upper triangle holds the symmetric entries */
            for (int i = 0; i < k; i++) a = a - L[j][i] * L[k][i];
            L[j][k] = a / x;
        }
    }
    double y[3] = {rhs[0], rhs[1], rhs[2]};
    for (int k = 0; k < 3; k++) { /* L y = rhs, column oriented */
        y[k] = y[k] / L[k][k];
        for (int j = k + 1; j < 3; j++) y[j] = y[j] - L[j][k] * y[k];
    }
    for (int k = 2; k >= 0; k--) { /* L^T z = y, column oriented */
        y[k] = y[k] / L[k][k];
        for (int j = 0; j < k; j++) y[j] = y[j] - L[k][j] * y[k];
    }
    z[0] = y[0]; z[1] = y[1]; z[2] = y[2];
    return 0;
}

/* DENSE_SCHUR solve of min |J y - r|^2 + |D y|^2 with e-block = column 0, f-blocks = 1..3 */
static int dense_schur(const double* J, const double* r, int n, const double D[4], double y[4])
{
    double S[3][3] = {{0}}, rhs[3] = {0, 0, 0};
    for (int k = 0; k < 3; k++) S[k][k] = S[k][k] + D[1 + k] * D[1 + k];
    double ete = D[0] * D[0], g = 0.0, buf[3] = {0, 0, 0};
    for (int i = 0; i < n; i++) {
        const double* row = J + 4 * (size_t)i;
        for (int a = 0; a < 3; a++)       /* EBlockRowOuterProduct: S += F'F (upper) */
            for (int b = a; b < 3; b++) S[a][b] = S[a][b] + row[1 + a] * row[1 + b];
        ete = ete + row[0] * row[0];
        g = g + row[0] * r[i];
        for (int a = 0; a < 3; a++) buf[a] = buf[a] + row[0] * row[1 + a];
    }
    const double inv = inv_psd1(ete);
    const double inv_g = inv * g;
    for (int i = 0; i < n; i++) {         /* UpdateRhs */
        const double* row = J + 4 * (size_t)i;
        const double sj = r[i] - row[0] * inv_g;
        for (int a = 0; a < 3; a++) rhs[a] = rhs[a] + row[1 + a] * sj;
    }
    for (int a = 0; a < 3; a++) {        /* ChunkOuterProduct: S -= (E'F)' inv (E'F) */
        const double bt = buf[a] * inv;
        for (int b = a; b < 3; b++) S[a][b] = S[a][b] - bt * buf[b];
    }
    double z[3];
    if (llt3_solve(S, rhs, z)) return -1;
    double ya = 0.0, ete2 = D[0] * D[0];  /* BackSubstitute */
    for (int i = 0; i < n; i++) {
        const double* row = J + 4 * (size_t)i;
        double sj = r[i];
        for (int a = 0; a < 3; a++) sj = sj - row[1 + a] * z[a];
        ya = ya + row[0] * sj;
        ete2 = ete2 + row[0] * row[0];
    }
    y[0] = inv_psd1(ete2) * ya;
    y[1] = z[0]; y[2] = z[1]; y[3] = z[2];
    return 0;
}

static double norm4(const double v[4])
{
    return sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3]);
}

/* The LM strategy's trust-region state (levenberg_marquardt_strategy.cc), factored out so it
 * can be held to Ceres' own unit tests (levenberg_marquardt_strategy_test.cc:81-110 radius
 * schedule, :113-160 diagonal handed to the linear solver; tests/test_oracle_lm.py). */
void pfo_lms_init(pfo_lm_strategy* s, double initial_radius, double max_radius, double min_diag,
                  double max_diag)
{ /* levenberg_marquardt_strategy.cc:47-61 */
    s->radius = initial_radius;
    s->max_radius = max_radius;
    s->decrease = 2.0;
    s->min_diag = min_diag;
    s->max_diag = max_diag;
    s->reuse_diag = 0;
    s->diag[0] = s->diag[1] = s->diag[2] = s->diag[3] = 0.0;
}

void pfo_lms_rejected(pfo_lm_strategy* s, double step_quality)
{ /* :156-160 (the quality is unused); an invalid step is rejected with quality 0 */
    (void)step_quality;
    s->radius = s->radius / s->decrease;
    s->decrease *= 2.0;
    s->reuse_diag = 1;
}

static void lms_accepted(pfo_lm_strategy* s, double step_quality, int use_pow)
{ /* :147-154: radius /= max(1/3, 1 - (2 q - 1)^3), capped at max_radius */
    const double q = 2.0 * step_quality - 1.0;
    const double f = 1.0 - (use_pow ? pow(q, 3) : q * q * q);
    s->radius = s->radius / (f > 1.0 / 3.0 ? f : 1.0 / 3.0);
    s->radius = s->radius < s->max_radius ? s->radius : s->max_radius;
    s->decrease = 2.0;
    s->reuse_diag = 0;
}

void pfo_lms_accepted(pfo_lm_strategy* s, double step_quality) { lms_accepted(s, step_quality, 1); }

void pfo_lms_regularizer(pfo_lm_strategy* s, const double* colsq, int n, double* D)
{ /* :75-88, :122: the diagonal = squared column norms of the (scaled) Jacobian clamped to
   * [min_lm_diagonal, max_lm_diagonal], recomputed only after an accepted step;
   * D = sqrt(diagonal / radius) goes to the linear solver as PerSolveOptions::D */
    if (!s->reuse_diag)
        for (int k = 0; k < n; k++) {
            const double d = colsq[k] > s->min_diag ? colsq[k] : s->min_diag;
            s->diag[k] = d < s->max_diag ? d : s->max_diag;
        }
    for (int k = 0; k < n; k++) D[k] = sqrt(s->diag[k] / s->radius);
    s->reuse_diag = 1;
}

int pfo_lm_fit(const double* xs, const double* ys, int n, double coef[4], pfo_lm_summary* sum)
{
    if (n <= 0) return -1;
    lm_problem P = {n, xs, ys, (double*)malloc(sizeof(double) * 4 * (size_t)n)};
    double* r = (double*)malloc(sizeof(double) * (size_t)n);
    double* mr = (double*)malloc(sizeof(double) * (size_t)n);
    if (!P.J || !r || !mr) { free(P.J); free(r); free(mr); return -1; }
    pfo_lm_summary s;
    memset(&s, 0, sizeof(s));
    double x[4] = {1.0, 1.0, 1.0, 1.0};  /* Depth.cpp:1270-1274 */
    double best[4] = {1.0, 1.0, 1.0, 1.0};
    double g[4], scale[4], colsq[4], D[4], step[4], delta[4], cand[4];
    pfo_lm_strategy lms;
    pfo_lms_init(&lms, LM_INIT_RADIUS, LM_MAX_RADIUS, LM_MIN_DIAG, LM_MAX_DIAG);
    int invalid_run = 0;
    double x_norm = -1.0;  /* trust_region_minimizer.cc:167: not set again until a step is accepted */

    /* iteration zero (:177-212, :226-279) */
    double x_cost = lm_evaluate(&P, x, r, P.J, g);
    col_sqnorm(P.J, n, scale);
    for (int k = 0; k < 4; k++) scale[k] = 1.0 / (1.0 + sqrt(scale[k]));
    for (int i = 0; i < n; i++)
        for (int k = 0; k < 4; k++) P.J[4 * (size_t)i + k] *= scale[k];
    s.initial_cost = x_cost;
    double min_cost = DBL_MAX;
    int iteration = 0, successful = 1, term = PFO_LM_NO_CONVERGENCE;
    double rel_decrease = 0.0, model_change = 0.0;
    for (;;) {
        /* FinalizeIterationAndCheckIfMinimizerCanContinue (:291-335) */
        if (successful) {
            s.successful++;
            if (x_cost < min_cost) { min_cost = x_cost; memcpy(best, x, sizeof(best)); }
        } else s.unsuccessful++;
        if (iteration >= LM_MAX_ITER) { term = PFO_LM_NO_CONVERGENCE; break; }
        if (successful) {
            double gmax = 0.0;
            for (int k = 0; k < 4; k++) {
                const double d = fabs(x[k] - (x[k] + -g[k]));
                if (d > gmax) gmax = d;
            }
            if (gmax <= LM_GRAD_TOL) { term = PFO_LM_GRADIENT_TOL; break; }
        }
        if (lms.radius <= LM_MIN_RADIUS) { term = PFO_LM_MIN_RADIUS; break; }
        iteration++;

        /* ComputeTrustRegionStep -> LevenbergMarquardtStrategy::ComputeStep (:355-424) */
        if (!lms.reuse_diag) col_sqnorm(P.J, n, colsq);
        pfo_lms_regularizer(&lms, colsq, 4, D);
        int ok = dense_schur(P.J, r, n, D, step) == 0;
        for (int k = 0; ok && k < 4; k++) ok = isfinite(step[k]);
        int valid = 0;
        if (ok) {
            for (int k = 0; k < 4; k++) step[k] = step[k] * -1.0;
            model_change = 0.0;
            double dot = 0.0;
            for (int i = 0; i < n; i++) {
                const double* row = P.J + 4 * (size_t)i;
                mr[i] = 0.0;
                for (int k = 0; k < 4; k++) mr[i] = mr[i] + row[k] * step[k];
            }
            for (int i = 0; i < n; i++) dot = dot + mr[i] * (r[i] + mr[i] / 2.0);
            model_change = -dot;
            valid = model_change > 0.0;
        }
        if (!valid) { /* HandleInvalidStep (:429-462) */
            if (++invalid_run >= LM_MAX_INVALID) { term = PFO_LM_FAILURE; break; }
            pfo_lms_rejected(&lms, 0.0);  /* StepIsInvalid = StepRejected(0) */
            successful = 0;
            continue;
        }
        invalid_run = 0;
        for (int k = 0; k < 4; k++) delta[k] = step[k] * scale[k];
        for (int k = 0; k < 4; k++) cand[k] = x[k] + delta[k];
        double cand_cost = lm_evaluate(&P, cand, NULL, NULL, NULL);
        if (!isfinite(cand_cost)) cand_cost = DBL_MAX;  /* :727-733 failed evaluation */
        /* ParameterToleranceReached (:667-685) */
        double dx[4];
        for (int k = 0; k < 4; k++) dx[k] = x[k] - cand[k];
        if (norm4(dx) <= LM_PARAM_TOL * (x_norm + LM_PARAM_TOL)) { term = PFO_LM_PARAMETER_TOL; break; }
        /* FunctionToleranceReached (:688-705) */
        if (fabs(x_cost - cand_cost) <= LM_FUNC_TOL * x_cost) { term = PFO_LM_FUNCTION_TOL; break; }
        /* IsStepSuccessful (:736-762) with the monotonic step evaluator */
        rel_decrease = (x_cost - cand_cost) / model_change;
        if (rel_decrease > LM_MIN_REL_DECREASE) { /* HandleSuccessfulStep (:767-779) */
            memcpy(x, cand, sizeof(x));
            x_norm = norm4(x);
            x_cost = lm_evaluate(&P, x, r, P.J, g);
            for (int i = 0; i < n; i++)
                for (int k = 0; k < 4; k++) P.J[4 * (size_t)i + k] *= scale[k];
            pfo_lms_accepted(&lms, rel_decrease);
            successful = 1;
        } else { /* HandleUnsuccessfulStep (:782-786) */
            pfo_lms_rejected(&lms, rel_decrease);
            successful = 0;
        }
    }
    memcpy(coef, best, sizeof(best));
    s.iterations = iteration;
    s.termination = term;
    s.final_cost = min_cost;
    if (sum) *sum = s;
    free(P.J);
    free(r);
    free(mr);
    return 0;
}

int pfo_register_tile_lm(const pfo_tile* t, const float* tiles, const float* emap, int ew,
                         int eh, int ec, float zr0, float zr1, double* coef64, float* abcd,
                         pfo_lm_summary* sum)
{ /* SolveDepthToDepth with one active map (Depth.cpp:1261-1414, driver :794-805) */
    int cols, rows;
    float zt, zd;
    int ns = pfo_reg_grid(t, zr0, zr1, &cols, &rows, &zt, &zd);
    if (cols <= 0 || rows <= 0) return -1;
    double* xs = (double*)malloc(sizeof(double) * ns);
    double* ys = (double*)malloc(sizeof(double) * ns);
    pfo_reg_samples(t, tiles, emap, ew, eh, ec, zr0, zr1, xs, ys);
    double c[4];
    int rc = pfo_lm_fit(xs, ys, ns, c, sum);
    free(xs);
    free(ys);
    if (rc) return rc;
    for (int i = 0; i < 4; i++) {
        if (coef64) coef64[i] = c[i];
        abcd[i] = (float)c[i];  /* abcd = Vec4f(vars[0..3]), Depth.cpp:1408 */
    }
    return 0;
}

int pfo_merge_lm(const float* emap, int ew, int eh, int ec, const pfo_tile* tiles, int ntiles,
                 float* tile_data, int out_w, float zr0, float zr1, uint16_t* out,
                 float* abcd_out)
{ /* MergeDepthMaps core (Depth.cpp:789-913) with the Ceres LM registration */
    for (int p = 0; p < ntiles; p++) {
        float abcd[4];
        if (pfo_register_tile_lm(&tiles[p], tile_data, emap, ew, eh, ec, zr0, zr1, NULL, abcd,
                                 NULL))
            return -2;
        pfo_depth_to_depth(&tiles[p], tile_data, abcd);
        if (abcd_out) memcpy(abcd_out + 4 * p, abcd, sizeof(abcd));
    }
    return pfo_solve_depth_all(emap, ew, eh, ec, tiles, ntiles, tile_data, out_w, out_w / 2,
                               zr0, zr1, out, NULL);
}

/* ------------------------------------------------------------------------------------------
 * The same Levenberg-Marquardt run evaluated from the 15 normal-equation moments of the samples
 * (the 14 sums of pf_oracle.c's reg_terms in its fixed 256-lane order, plus sum y^2) instead of a
 * pass over the samples per evaluation: the residual problem is linear, so cost, gradient, J'J
 * and every quantity above are exact functions of the moments.  This is the form the HIP
 * registration kernel runs (pf_kernels.hip lm_moments, bit-identical: only +, -, *, /, sqrt);
 * it departs from the sample-wise restatement above by rounding only (cost as 0.5 (y'y - 2 p'J'y
 * + p'J'J p), pow(q, 3) as q*q*q), which tests/test_oracle_lm.py bounds.
 *   M = [[S0,S1,S2,S3],[S1,S4,S5,S6],[S2,S5,S7,S8],[S3,S6,S8,S9]] = J'J,  Jy = S10..S13,
 *   yy = S14. */
static double mom_cost(const double S[15], const double p[4])
{
    const double M[4][4] = {{S[0], S[1], S[2], S[3]}, {S[1], S[4], S[5], S[6]},
                            {S[2], S[5], S[7], S[8]}, {S[3], S[6], S[8], S[9]}};
    double pMp = 0.0, pJy = 0.0;
    for (int i = 0; i < 4; i++) {
        double q = 0.0;
        for (int j = 0; j < 4; j++) q = q + M[i][j] * p[j];
        pMp = pMp + p[i] * q;
        pJy = pJy + p[i] * S[10 + i];
    }
    return 0.5 * ((S[14] - 2.0 * pJy) + pMp);
}

static void mom_gradient(const double S[15], const double p[4], double g[4])
{
    const double M[4][4] = {{S[0], S[1], S[2], S[3]}, {S[1], S[4], S[5], S[6]},
                            {S[2], S[5], S[7], S[8]}, {S[3], S[6], S[8], S[9]}};
    for (int i = 0; i < 4; i++) {
        double q = 0.0;
        for (int j = 0; j < 4; j++) q = q + M[i][j] * p[j];
        g[i] = q - S[10 + i];
    }
}

int pfo_lm_moments(const double S[15], double coef[4], pfo_lm_summary* sum)
{
    const double M[4][4] = {{S[0], S[1], S[2], S[3]}, {S[1], S[4], S[5], S[6]},
                            {S[2], S[5], S[7], S[8]}, {S[3], S[6], S[8], S[9]}};
    pfo_lm_summary s;
    memset(&s, 0, sizeof(s));
    double x[4] = {1.0, 1.0, 1.0, 1.0}, best[4] = {1.0, 1.0, 1.0, 1.0};
    double sc[4], Ms[4][4], g[4], gs[4], colsq[4], D[4], step[4], cand[4];
    for (int k = 0; k < 4; k++) sc[k] = 1.0 / (1.0 + sqrt(M[k][k]));
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) Ms[i][j] = (M[i][j] * sc[i]) * sc[j];
    double x_norm = -1.0;
    pfo_lm_strategy lms;
    pfo_lms_init(&lms, LM_INIT_RADIUS, LM_MAX_RADIUS, LM_MIN_DIAG, LM_MAX_DIAG);
    int invalid_run = 0;
    double x_cost = mom_cost(S, x);
    mom_gradient(S, x, g);
    s.initial_cost = x_cost;
    double min_cost = DBL_MAX;
    int iteration = 0, successful = 1, term = PFO_LM_NO_CONVERGENCE;
    for (;;) {
        if (successful) {
            s.successful++;
            if (x_cost < min_cost) { min_cost = x_cost; memcpy(best, x, sizeof(best)); }
        } else s.unsuccessful++;
        if (iteration >= LM_MAX_ITER) { term = PFO_LM_NO_CONVERGENCE; break; }
        if (successful) {
            double gmax = 0.0;
            for (int k = 0; k < 4; k++) {
                const double d = fabs(x[k] - (x[k] + -g[k]));
                if (d > gmax) gmax = d;
            }
            if (gmax <= LM_GRAD_TOL) { term = PFO_LM_GRADIENT_TOL; break; }
        }
        if (lms.radius <= LM_MIN_RADIUS) { term = PFO_LM_MIN_RADIUS; break; }
        iteration++;
        for (int k = 0; k < 4; k++) colsq[k] = Ms[k][k];
        pfo_lms_regularizer(&lms, colsq, 4, D);
        for (int k = 0; k < 4; k++) gs[k] = sc[k] * g[k];  /* J_s' r */
        /* Schur elimination of column 0 (as dense_schur above, from the moments) */
        double ete = D[0] * D[0] + Ms[0][0];
        double R[3][3], rhs[3], z[3];
        for (int a = 0; a < 3; a++)
            for (int b = a; b < 3; b++)
                R[a][b] = Ms[1 + a][1 + b] + (a == b ? D[1 + a] * D[1 + a] : 0.0);
        const double inv = inv_psd1(ete);
        const double inv_g = inv * gs[0];
        for (int a = 0; a < 3; a++) rhs[a] = gs[1 + a] - Ms[0][1 + a] * inv_g;
        for (int a = 0; a < 3; a++) {
            const double bt = Ms[0][1 + a] * inv;
            for (int b = a; b < 3; b++) R[a][b] = R[a][b] - bt * Ms[0][1 + b];
        }
        int ok = llt3_solve(R, rhs, z) == 0;
        if (ok) {
            double ya = gs[0];
            for (int a = 0; a < 3; a++) ya = ya - Ms[0][1 + a] * z[a];
            step[0] = inv * ya;
            step[1] = z[0]; step[2] = z[1]; step[3] = z[2];
            for (int k = 0; ok && k < 4; k++) ok = isfinite(step[k]);
        }
        int valid = 0;
        double mcc = 0.0;
        if (ok) {
            for (int k = 0; k < 4; k++) step[k] = step[k] * -1.0;
            /* -(J s).(r + J s / 2) = -(s.J'r + s.J'J s / 2) */
            double sJr = 0.0, sMs = 0.0;
            for (int i = 0; i < 4; i++) {
                double q = 0.0;
                for (int j = 0; j < 4; j++) q = q + Ms[i][j] * step[j];
                sMs = sMs + step[i] * q;
                sJr = sJr + step[i] * gs[i];
            }
            mcc = -(sJr + sMs / 2.0);
            valid = mcc > 0.0;
        }
        if (!valid) {
            if (++invalid_run >= LM_MAX_INVALID) { term = PFO_LM_FAILURE; break; }
            pfo_lms_rejected(&lms, 0.0);
            successful = 0;
            continue;
        }
        invalid_run = 0;
        for (int k = 0; k < 4; k++) cand[k] = x[k] + step[k] * sc[k];
        double cand_cost = mom_cost(S, cand);
        if (!isfinite(cand_cost)) cand_cost = DBL_MAX;
        double dx[4];
        for (int k = 0; k < 4; k++) dx[k] = x[k] - cand[k];
        if (norm4(dx) <= LM_PARAM_TOL * (x_norm + LM_PARAM_TOL)) { term = PFO_LM_PARAMETER_TOL; break; }
        if (fabs(x_cost - cand_cost) <= LM_FUNC_TOL * x_cost) { term = PFO_LM_FUNCTION_TOL; break; }
        const double rel = (x_cost - cand_cost) / mcc;
        if (rel > LM_MIN_REL_DECREASE) {
            memcpy(x, cand, sizeof(x));
            x_norm = norm4(x);
            x_cost = mom_cost(S, x);
            mom_gradient(S, x, g);
            lms_accepted(&lms, rel, 0);  /* (2 rel - 1)^3 as q*q*q, as the GPU */
            successful = 1;
        } else {
            pfo_lms_rejected(&lms, rel);
            successful = 0;
        }
    }
    memcpy(coef, best, sizeof(best));
    s.iterations = iteration;
    s.termination = term;
    s.final_cost = min_cost;
    if (sum) *sum = s;
    return 0;
}
