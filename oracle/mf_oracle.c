/*
 * mf_oracle.c -- CPU restatement of the reference SGD path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product path (the
 * `matrix_factorization` package or libmf_hip.so) links, loads or calls this
 * file.  It is imported only by tests/, __graft_entry__.smoke() and the
 * `cpu_baseline` leg of bench.py, always as the checker / reported baseline.
 *
 * Parity anchor: pinned against golden vectors produced by the reference's
 * own Python source (tests/golden/make_golden.py), see DESIGN.md section 3.
 *
 * Every function follows the reference line by line, in FP64, with the
 * reference's addition order and with FP contraction disabled
 * (-ffp-contract=off), so that each scalar expression rounds exactly as the
 * numba / CPython evaluation of the same expression does.  The one place the
 * reference's order is not pinned is the k-long dot product (np.dot -> BLAS
 * ddot, kernels.py:43,74,152,227) and np.sum of squares (kernels.py:102,302):
 * here they are summed sequentially f = 0..k-1.
 *
 * Reference files (all under /root/reference/matrix_factorization/):
 *   kernels.py                     per-rating predictors and SGD updates
 *   kernel_matrix_factorization.py _calculate_rmse / _sgd / _predict
 *   baseline_model.py              bias-only SGD / ALS (BaselineModel)
 */
#include <math.h>
#include <stdint.h>
#include <stddef.h>

enum { OR_LINEAR = 0, OR_SIGMOID = 1, OR_RBF = 2 };

/* kernels.py:6-18 */
static double or_sigmoid(double x) { return 1.0 / (1.0 + exp(-x)); }

static double or_dot(const double* p, const double* q, int32_t k) {
    double s = 0.0;
    for (int32_t f = 0; f < k; ++f) s += p[f] * q[f];
    return s;
}

static double or_sqdist(const double* p, const double* q, int32_t k) {
    double s = 0.0;
    for (int32_t f = 0; f < k; ++f) {
        double d = p[f] - q[f];
        s += d * d;
    }
    return s;
}

/* Predictors: kernels.py:21-45 (linear), :48-78 (sigmoid), :81-105 (rbf). */
static double or_predict_one(int32_t kernel, double mu, double bu, double bi,
                             const double* p, const double* q, int32_t k,
                             double gamma, double a, double c) {
    if (kernel == OR_LINEAR) {
        return ((mu + bi) + bu) + or_dot(p, q, k);          /* kernels.py:42-44 */
    } else if (kernel == OR_SIGMOID) {
        double x = ((mu + bu) + bi) + or_dot(p, q, k);      /* kernels.py:73-75 */
        return a + c * or_sigmoid(x);                        /* kernels.py:76-77 */
    } else {
        double power = (-gamma) * or_sqdist(p, q, k);        /* kernels.py:102 */
        return a + c * exp(power);                           /* kernels.py:103-104 */
    }
}

/*
 * One sequential SGD sweep: kernel_matrix_factorization.py:374-425 with the
 * per-rating bodies of kernels.py:108-180 (linear), :183-262 (sigmoid) and
 * :265-327 (rbf).  `order` (nullable) lists the rating indices in visit
 * order, i.e. the row order of X after `np.random.shuffle(X)` (:371).
 * a = min_rating, c = max_rating - min_rating (:405-406, :420-421).
 */
int oracle_sgd_pass(const int32_t* uid, const int32_t* iid, const double* r,
                    int64_t n, const int64_t* order, double mu,
                    double* bu, double* bi, double* P, double* Q, int32_t k,
                    int32_t kernel, double gamma, double lr, double reg,
                    double a, double c, int32_t upd_user, int32_t upd_item) {
    for (int64_t t = 0; t < n; ++t) {
        int64_t j = order ? order[t] : t;
        int64_t u = uid[j], it = iid[j];
        double rating = r[j];
        double* p = P + u * (int64_t)k;
        double* q = Q + it * (int64_t)k;
        if (kernel == OR_LINEAR) {
            double ub = bu[u], ib = bi[it];                  /* kernels.py:144-145 */
            double pred = ((mu + ib) + ub) + or_dot(p, q, k); /* :148-153 */
            double e = pred - rating;                         /* :156 */
            if (upd_user) bu[u] = bu[u] - lr * (e + reg * ub);  /* :159-160 */
            if (upd_item) bi[it] = bi[it] - lr * (e + reg * ib); /* :162-163 */
            for (int32_t f = 0; f < k; ++f) {                 /* :166-178 */
                double pf = p[f], qf = q[f];
                if (upd_user) p[f] = p[f] - lr * (e * qf + reg * pf);
                if (upd_item) q[f] = q[f] - lr * (e * pf + reg * qf);
            }
        } else if (kernel == OR_SIGMOID) {
            double ub = bu[u], ib = bi[it];                  /* kernels.py:220-221 */
            double x = ((mu + ub) + ib) + or_dot(p, q, k);   /* :226-228 */
            double s = or_sigmoid(x);                         /* :229 */
            double pred = a + c * s;                          /* :230 */
            double e = pred - rating;                         /* :233 */
            double d = (s * s) * exp(-x);                     /* :236 (no c factor) */
            if (upd_user) bu[u] = bu[u] - lr * (e * d + reg * ub);  /* :239-241 */
            if (upd_item) bi[it] = bi[it] - lr * (e * d + reg * ib); /* :243-245 */
            for (int32_t f = 0; f < k; ++f) {                 /* :248-260 */
                double pf = p[f], qf = q[f];
                if (upd_user) p[f] = p[f] - lr * (e * (qf * d) + reg * pf);
                if (upd_item) q[f] = q[f] - lr * (e * (pf * d) + reg * qf);
            }
        } else {
            double power = (-gamma) * or_sqdist(p, q, k);    /* kernels.py:302 */
            double E = exp(power);                            /* :303 */
            double pred = a + c * E;                          /* :304 */
            double e = pred - rating;                         /* :307 */
            double d = (2.0 * E) * gamma;                     /* :310 (no c factor) */
            for (int32_t f = 0; f < k; ++f) {                 /* :313-325 */
                double pf = p[f], qf = q[f];
                if (upd_user) p[f] = p[f] - lr * (e * (d * (qf - pf)) + reg * pf);
                if (upd_item) q[f] = q[f] - lr * (e * (d * (pf - qf)) + reg * qf);
            }
        }
    }
    return 0;
}

/* kernel_matrix_factorization.py:240-317: sum of squared (r - pred), then
 * sqrt(mean).  Returned as the sum of squares so callers can combine shards;
 * rmse = sqrt(sse / n). */
double oracle_sse(const int32_t* uid, const int32_t* iid, const double* r,
                  int64_t n, double mu, const double* bu, const double* bi,
                  const double* P, const double* Q, int32_t k, int32_t kernel,
                  double gamma, double a, double c) {
    double sse = 0.0;
    for (int64_t j = 0; j < n; ++j) {
        int64_t u = uid[j], it = iid[j];
        double pred = or_predict_one(kernel, mu, bu[u], bi[it],
                                     P + u * (int64_t)k, Q + it * (int64_t)k,
                                     k, gamma, a, c);
        double err = r[j] - pred;                             /* :313 */
        sse += err * err;
    }
    return sse;
}

/* kernel_matrix_factorization.py:448-541.  Ids of -1 mean "unknown": bias 0
 * and an all-zero factor vector (:487-499).  Clipped when bound != 0. */
void oracle_predict(const int32_t* uid, const int32_t* iid, int64_t n,
                    double mu, const double* bu, const double* bi,
                    const double* P, const double* Q, int32_t k,
                    int32_t kernel, double gamma, double min_rating,
                    double max_rating, int32_t bound, double* out,
                    double* zeros /* k doubles of scratch, zeroed */) {
    for (int32_t f = 0; f < k; ++f) zeros[f] = 0.0;
    double a = min_rating, c = max_rating - min_rating;
    for (int64_t j = 0; j < n; ++j) {
        int64_t u = uid[j], it = iid[j];
        int uk = u != -1, ik = it != -1;
        double ub = uk ? bu[u] : 0.0;
        double ib = ik ? bi[it] : 0.0;
        const double* p = uk ? P + u * (int64_t)k : zeros;
        const double* q = ik ? Q + it * (int64_t)k : zeros;
        double pred = or_predict_one(kernel, mu, ub, ib, p, q, k, gamma, a, c);
        if (bound) {                                          /* :532-536 */
            if (pred > max_rating) pred = max_rating;
            else if (pred < min_rating) pred = min_rating;
        }
        out[j] = pred;
    }
}

/* ---- BaselineModel (bias only), baseline_model.py ---------------------- */

/* baseline_model.py:255-266 */
int oracle_bias_sgd_pass(const int32_t* uid, const int32_t* iid,
                         const double* r, int64_t n, const int64_t* order,
                         double mu, double* bu, double* bi, double lr,
                         double reg, int32_t upd_user, int32_t upd_item) {
    for (int64_t t = 0; t < n; ++t) {
        int64_t j = order ? order[t] : t;
        int64_t u = uid[j], it = iid[j];
        double pred = (mu + bu[u]) + bi[it];                  /* :259 */
        double err = r[j] - pred;                             /* :260 */
        if (upd_user) bu[u] = bu[u] + lr * (err - reg * bu[u]);    /* :264 */
        if (upd_item) bi[it] = bi[it] + lr * (err - reg * bi[it]); /* :266 */
    }
    return 0;
}

/* baseline_model.py:183-212 (sum of squares; rmse = sqrt(sse/n)) */
double oracle_bias_sse(const int32_t* uid, const int32_t* iid, const double* r,
                       int64_t n, double mu, const double* bu,
                       const double* bi) {
    double sse = 0.0;
    for (int64_t j = 0; j < n; ++j) {
        double pred = (mu + bu[uid[j]]) + bi[iid[j]];         /* :207 */
        double err = r[j] - pred;
        sse += err * err;
    }
    return sse;
}

/* One ALS epoch, baseline_model.py:326-348.  ucnt/icnt are the per-id rating
 * counts (:317-323) as doubles; bu/bi are overwritten. */
int oracle_bias_als_epoch(const int32_t* uid, const int32_t* iid,
                          const double* r, int64_t n, double mu, double* bu,
                          double* bi, const double* ucnt, const double* icnt,
                          int32_t n_users, int32_t n_items, double reg) {
    for (int32_t u = 0; u < n_users; ++u) bu[u] = 0.0;        /* :329 */
    for (int64_t j = 0; j < n; ++j)                           /* :332-334 */
        bu[uid[j]] += (r[j] - mu) - bi[iid[j]];
    for (int32_t u = 0; u < n_users; ++u) bu[u] = bu[u] / (reg + ucnt[u]); /* :337 */
    for (int32_t i = 0; i < n_items; ++i) bi[i] = 0.0;        /* :340 */
    for (int64_t j = 0; j < n; ++j)                           /* :343-345 */
        bi[iid[j]] += (r[j] - mu) - bu[uid[j]];
    for (int32_t i = 0; i < n_items; ++i) bi[i] = bi[i] / (reg + icnt[i]); /* :348 */
    return 0;
}
