/*
 * lqro_oracle.c — TEST INFRASTRUCTURE ONLY (see lqro_oracle.h).
 *
 * Plain-C restatement of the reference's per-timestep LQR-Obstacle path.
 * Compiled with -O2 -ffp-contract=off (no FMA contraction, IEEE double/float,
 * SSE on x86-64) so that every arithmetic operation rounds exactly where the
 * reference's g++ build does.  Operation ORDER follows the reference line by
 * line: Matrix products accumulate from 0.0 in k order (MAT:218-231), C++
 * expression chains associate left to right, unary minus binds first.
 */
#include "lqro_oracle.h"
#include "lqro_qhull.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <time.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int orc_version(void) { return 1; }

/* ------------------------------------------------------------------------ */
/* Fixed-size fp64 matrix helpers, row-major, MAT semantics.                 */
/* ------------------------------------------------------------------------ */
#define MXN 16

/* out = a(r x k) * b(k x c); temp accumulates from 0 in k order (MAT:218-231) */
static void mm(int r, int k, int c, const double* a, const double* b, double* out) {
  double t[MXN * MXN];
  for (int i = 0; i < r; ++i)
    for (int j = 0; j < c; ++j) {
      double temp = 0.0;
      for (int kk = 0; kk < k; ++kk) temp += a[i * k + kk] * b[kk * c + j];
      t[i * c + j] = temp;
    }
  memcpy(out, t, sizeof(double) * (size_t)(r * c));
}
/* out = ~a  (MAT:238-246) */
static void mt(int r, int c, const double* a, double* out) {
  double t[MXN * MXN];
  for (int i = 0; i < c; ++i)
    for (int j = 0; j < r; ++j) t[i * r + j] = a[j * c + i];
  memcpy(out, t, sizeof(double) * (size_t)(r * c));
}
static void madd(int n, const double* a, const double* b, double* out) {
  for (int i = 0; i < n; ++i) out[i] = a[i] + b[i];
}
static void msub(int n, const double* a, const double* b, double* out) {
  for (int i = 0; i < n; ++i) out[i] = a[i] - b[i];
}
/* Matrix*double and double*Matrix both compute elem*a (MAT:196-201, 261) */
static void mscale(int n, const double* a, double s, double* out) {
  for (int i = 0; i < n; ++i) out[i] = a[i] * s;
}
static void mneg(int n, const double* a, double* out) {
  for (int i = 0; i < n; ++i) out[i] = -a[i];
}
static void meye(int n, double* out) {
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) out[i * n + j] = (i == j ? 1.0 : 0.0);
}

/* operator! : full-pivot Gauss-Jordan inverse (MAT:603-671) */
static void minv(int n, const double* q, double* out) {
  double m[MXN * MXN], inv[MXN * MXN];
  size_t row_p[MXN], col_p[MXN];
  memcpy(m, q, sizeof(double) * (size_t)(n * n));
  meye(n, inv);
  for (int i = 0; i < n; ++i) { row_p[i] = (size_t)i; col_p[i] = (size_t)i; }
  for (int k = 0; k < n; ++k) {
    double maximum = 0.0; int max_row = k, max_col = k;
    for (int i = k; i < n; ++i)
      for (int j = k; j < n; ++j) {
        double abs_ij = fabs(m[row_p[i] * n + col_p[j]]);
        if (abs_ij > maximum) { maximum = abs_ij; max_row = i; max_col = j; }
      }
    size_t sw = row_p[k]; row_p[k] = row_p[max_row]; row_p[max_row] = sw;
    sw = col_p[k]; col_p[k] = col_p[max_col]; col_p[max_col] = sw;
    for (int i = k + 1; i < n; ++i) {
      double factor = m[row_p[i] * n + col_p[k]] / m[row_p[k] * n + col_p[k]];
      for (int j = k + 1; j < n; ++j)
        m[row_p[i] * n + col_p[j]] -= factor * m[row_p[k] * n + col_p[j]];
      for (int j = 0; j < k; ++j)
        inv[row_p[i] * n + row_p[j]] -= factor * inv[row_p[k] * n + row_p[j]];
      inv[row_p[i] * n + row_p[k]] = -factor;
    }
  }
  for (int k = n - 1; k >= 0; --k) {
    double quotient = m[row_p[k] * n + col_p[k]];
    for (int j = 0; j < n; ++j) inv[row_p[k] * n + j] /= quotient;
    for (int i = 0; i < k; ++i) {
      double factor = m[row_p[i] * n + col_p[k]];
      for (int j = 0; j < n; ++j) inv[row_p[i] * n + j] -= factor * inv[row_p[k] * n + j];
    }
  }
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) m[col_p[i] * n + j] = inv[row_p[i] * n + j];
  memcpy(out, m, sizeof(double) * (size_t)(n * n));
}

/* operator% : solve P X = Q, full pivoting (MAT:370-442) */
static void msolve(int n, int nc, const double* p, const double* q, double* out) {
  double m[MXN * MXN], inv[MXN * MXN];
  size_t row_p[MXN], col_p[MXN], invrow_p[MXN];
  memcpy(m, p, sizeof(double) * (size_t)(n * n));
  memcpy(inv, q, sizeof(double) * (size_t)(n * nc));
  for (int i = 0; i < n; ++i) { row_p[i] = (size_t)i; col_p[i] = (size_t)i; }
  for (int k = 0; k < n; ++k) {
    double maximum = 0.0; int max_row = k, max_col = k;
    for (int i = k; i < n; ++i)
      for (int j = k; j < n; ++j) {
        double abs_ij = fabs(m[row_p[i] * n + col_p[j]]);
        if (abs_ij > maximum) { maximum = abs_ij; max_row = i; max_col = j; }
      }
    size_t sw = row_p[k]; row_p[k] = row_p[max_row]; row_p[max_row] = sw;
    sw = col_p[k]; col_p[k] = col_p[max_col]; col_p[max_col] = sw;
    for (int i = k + 1; i < n; ++i) {
      double factor = m[row_p[i] * n + col_p[k]] / m[row_p[k] * n + col_p[k]];
      for (int j = k + 1; j < n; ++j)
        m[row_p[i] * n + col_p[j]] -= factor * m[row_p[k] * n + col_p[j]];
      for (int j = 0; j < nc; ++j) inv[row_p[i] * nc + j] -= factor * inv[row_p[k] * nc + j];
    }
  }
  for (int k = n - 1; k >= 0; --k) {
    double quotient = m[row_p[k] * n + col_p[k]];
    for (int j = 0; j < nc; ++j) inv[row_p[k] * nc + j] /= quotient;
    for (int i = 0; i < k; ++i) {
      double factor = m[row_p[i] * n + col_p[k]];
      for (int j = 0; j < nc; ++j) inv[row_p[i] * nc + j] -= factor * inv[row_p[k] * nc + j];
    }
  }
  for (int i = 0; i < n; ++i) invrow_p[row_p[i]] = (size_t)i;
  for (int i = 0; i < n; ++i) {
    for (int j = 0; j < nc; ++j) {
      double t = inv[col_p[i] * nc + j];
      inv[col_p[i] * nc + j] = inv[row_p[i] * nc + j];
      inv[row_p[i] * nc + j] = t;
    }
    row_p[invrow_p[col_p[i]]] = row_p[i];
    invrow_p[row_p[i]] = invrow_p[col_p[i]];
  }
  memcpy(out, inv, sizeof(double) * (size_t)(n * nc));
}

/* matrix 1-norm (MAT:273-286) */
static double mnorm1(int n, const double* q) {
  double norm1 = 0.0;
  for (int j = 0; j < n; ++j) {
    double colabssum = 0.0;
    for (int i = 0; i < n; ++i) colabssum += fabs(q[i * n + j]);
    if (colabssum > norm1) norm1 = colabssum;
  }
  return norm1;
}

/* exp: Pade-7 with scaling and squaring (MAT:763-790) */
static void mexp(int n, const double* q, double* out) {
  const double JB0 = 1729728e1, JB1 = 864864e1, JB2 = 199584e1, JB3 = 2772e2,
               JB4 = 252e2, JB5 = 1512e0, JB6 = 56e0, JB7 = 1e0;
  const double NORMLIM = 9.504178996162932e-1;
  double A[MXN * MXN], A2[MXN * MXN], A4[MXN * MXN], A6[MXN * MXN];
  double t1[MXN * MXN], t2[MXN * MXN], I[MXN * MXN], U[MXN * MXN], V[MXN * MXN];
  const int nn = n * n;
  memcpy(A, q, sizeof(double) * (size_t)nn);
  double l2 = ceil(log(mnorm1(n, A) / NORMLIM) * M_LOG2E);
  int s = (int)(0.0 < l2 ? l2 : 0.0); /* std::max(double(0), x): x if !(0 < x) is false */
  {
    double p = pow(2.0, s);
    for (int i = 0; i < nn; ++i) A[i] /= p;
  }
  mm(n, n, n, A, A, A2);
  mm(n, n, n, A2, A2, A4);
  mm(n, n, n, A2, A4, A6);
  meye(n, I);
  /* U = A*(A6*JB7 + A4*JB5 + A2*JB3 + I*JB1) */
  mscale(nn, A6, JB7, t1);
  mscale(nn, A4, JB5, t2); madd(nn, t1, t2, t1);
  mscale(nn, A2, JB3, t2); madd(nn, t1, t2, t1);
  mscale(nn, I, JB1, t2);  madd(nn, t1, t2, t1);
  mm(n, n, n, A, t1, U);
  /* V = A6*JB6 + A4*JB4 + A2*JB2 + I*JB0 */
  mscale(nn, A6, JB6, V);
  mscale(nn, A4, JB4, t2); madd(nn, V, t2, V);
  mscale(nn, A2, JB2, t2); madd(nn, V, t2, V);
  mscale(nn, I, JB0, t2);  madd(nn, V, t2, V);
  msub(nn, V, U, t1);
  madd(nn, V, U, t2);
  msolve(n, n, t1, t2, out);
  for (int i = 0; i < s; ++i) mm(n, n, n, out, out, out);
}

/* ------------------------------------------------------------------------ */
/* Model + gains: LQRO:167-189, 368-397, 421-471, 520-582, stdafx.h:76-96.   */
/* ------------------------------------------------------------------------ */
void orc_model_default(lqro_model* m) {
  m->dt = 1.0 / 30.0;                 /* LQRO:169 */
  m->gravity = 9.80665;               /* LQRO:170 */
  m->mass = 0.500;                    /* LQRO:177 */
  m->inertia = 0.1;                   /* LQRO:178 (inertia = 0.1*I3) */
  m->moment_const = 1.5e-9 / 6.11e-8; /* LQRO:179 */
  m->thrust_latency = 40.0;           /* LQRO:181 */
  m->length = 0.3429 / 2;             /* LQRO:182 */
  m->j_step = 0.0009765625;           /* LQRO:189 */
  m->qv = 100;                        /* LQRO:1278 */
  m->qp = 0.1;                        /* LQRO:1281 */
  m->r = 5;                           /* LQRO:1283 */
  m->pos_weight = 0.05;               /* LQRO:559-561 */
}

/* stdafx.h:76-84 */
static void skew(const double* v, double* out) {
  for (int i = 0; i < 9; ++i) out[i] = 0.0;
  out[0 * 3 + 1] = -v[2]; out[0 * 3 + 2] = v[1];
  out[1 * 3 + 0] = v[2];  out[1 * 3 + 2] = -v[0];
  out[2 * 3 + 0] = -v[1]; out[2 * 3 + 1] = v[0];
}
/* stdafx.h:86-96 */
static double hypot3(const double* v) {
  double X = fabs(v[0]), Y = fabs(v[1]), Z = fabs(v[2]);
  if (X > Y && X > Z) return X * sqrt(1.0 + (Y / X) * (Y / X) + (Z / X) * (Z / X));
  else if (Y > Z) return Y * sqrt(1.0 + (X / Y) * (X / Y) + (Z / Y) * (Z / Y));
  else return Z * sqrt(1.0 + (X / Z) * (X / Z) + (Y / Z) * (Y / Z));
}

typedef struct {
  double dt, gravity, mass, momentConst, thrust_latency, length, jStep;
  double inertia[9], invInertia[9];
} phys_t;

static void phys_init(const lqro_model* m, phys_t* p) {
  p->dt = m->dt; p->gravity = m->gravity; p->mass = m->mass;
  p->momentConst = m->moment_const; p->thrust_latency = m->thrust_latency;
  p->length = m->length; p->jStep = m->j_step;
  double I3[9]; meye(3, I3);
  mscale(9, I3, m->inertia, p->inertia);      /* 0.1*identity<3>() */
  minv(3, p->inertia, p->invInertia);         /* LQRO:187 */
}

/* f (LQRO:368-397).  X=16: the reference.  X=12: BASELINE config 5's reduced
 * model — no rotor-force states, F = u (not in the reference;
 * its restatement here pins the GPU's lqro_synthesize_gains_batch_x). */
static void fdyn_x(int X, const phys_t* P, const double* x, const double* R, const double* u, double* xdot);
static void fdyn(const phys_t* P, const double* x, const double* R, const double* u, double* xdot) {
  fdyn_x(16, P, x, R, u, xdot);
}
static void fdyn_x(int X, const phys_t* P, const double* x, const double* R, const double* u, double* xdot) {
  const double eX[3] = {1, 0, 0}, eY[3] = {0, 1, 0}, eZ[3] = {0, 0, 1};
  double v[3] = {x[3], x[4], x[5]}, r[3] = {x[6], x[7], x[8]}, w[3] = {x[9], x[10], x[11]};
  double F[4];
  for (int i = 0; i < 4; ++i) F[i] = X == 16 ? x[12 + i] : u[i];
  double t3[3], t3b[3], S[9], E[9], RE[9];
  /* p_dot = v */
  xdot[0] = v[0]; xdot[1] = v[1]; xdot[2] = v[2];
  /* v_dot = -gravity*eZ + R*exp(skew(r))*((F0+F1+F2+F3)/mass)*eZ */
  double a[3];
  mscale(3, eZ, -P->gravity, a);
  skew(r, S); mexp(3, S, E);
  mm(3, 3, 3, R, E, RE);
  mscale(9, RE, (F[0] + F[1] + F[2] + F[3]) / P->mass, RE);
  mm(3, 3, 1, RE, eZ, t3);
  madd(3, a, t3, t3);
  xdot[3] = t3[0]; xdot[4] = t3[1]; xdot[5] = t3[2];
  /* r_dot */
  double l = hypot3(r);
  double S5[9], b[3];
  skew(r, S); mscale(9, S, 0.5, S5); mm(3, 3, 1, S5, w, b); madd(3, w, b, t3); /* w + 0.5*[r]*w */
  if (0.5 * l > 0.0) {
    double rl[3] = {r[0] / l, r[1] / l, r[2] / l}, Sl[9], Slw[3], c[3];
    skew(rl, Sl);
    mm(3, 3, 1, Sl, w, Slw);
    double sc = (1.0 - 0.5 * l / tan(0.5 * l));
    double ScSl[9];
    mscale(9, Sl, sc, ScSl);
    mm(3, 3, 1, ScSl, Slw, c);
    madd(3, t3, c, t3);
  }
  xdot[6] = t3[0]; xdot[7] = t3[1]; xdot[8] = t3[2];
  /* w_dot = invInertia*( l*(F1-F3)*eX + l*(F2-F0)*eY + (F0-F1+F2-F3)*kM*eZ - [w]*J*w ) */
  double s1[3], s2[3], s3[3], Sw[9], SwJ[9], s4[3];
  mscale(3, eX, P->length * (F[1] - F[3]), s1);
  mscale(3, eY, P->length * (F[2] - F[0]), s2);
  mscale(3, eZ, (F[0] - F[1] + F[2] - F[3]) * P->momentConst, s3);
  skew(w, Sw); mm(3, 3, 3, Sw, P->inertia, SwJ); mm(3, 3, 1, SwJ, w, s4);
  madd(3, s1, s2, t3b); madd(3, t3b, s3, t3b); msub(3, t3b, s4, t3b);
  mm(3, 3, 1, P->invInertia, t3b, t3);
  xdot[9] = t3[0]; xdot[10] = t3[1]; xdot[11] = t3[2];
  /* f_dot = latency*(u - F) */
  if (X == 16)
    for (int i = 0; i < 4; ++i) xdot[12 + i] = (u[i] - F[i]) * P->thrust_latency;
}

/* linearizeDiscretize (LQRO:456-471) with Jacobian_fx/fu (LQRO:421-441) */
static void linearize(int X, const phys_t* P, const double* x, const double* R, const double* u,
                      double* A, double* B, double* c) {
  enum { XM = 16, U = 4 };
  double F[XM * XM], G[XM * U], xdot[XM], fr[XM], fl[XM];
  double xr[XM], xl[XM], ur[U], ul[U];
  memcpy(xr, x, sizeof(double) * X); memcpy(xl, x, sizeof(double) * X);
  for (int i = 0; i < X; ++i) {
    xr[i] += P->jStep; xl[i] -= P->jStep;
    fdyn_x(X, P, xr, R, u, fr); fdyn_x(X, P, xl, R, u, fl);
    for (int k = 0; k < X; ++k) F[k * X + i] = (fr[k] - fl[k]) / (2 * P->jStep);
    xr[i] = xl[i] = x[i];
  }
  memcpy(ur, u, sizeof ur); memcpy(ul, u, sizeof ul);
  for (int i = 0; i < U; ++i) {
    ur[i] += P->jStep; ul[i] -= P->jStep;
    fdyn_x(X, P, x, R, ur, fr); fdyn_x(X, P, x, R, ul, fl);
    for (int k = 0; k < X; ++k) G[k * U + i] = (fr[k] - fl[k]) / (2 * P->jStep);
    ur[i] = ul[i] = u[i];
  }
  fdyn_x(X, P, x, R, u, xdot);
  double dtF[XM * XM], hF[XM * XM], E2[XM * XM], Int[XM * XM], I[XM * XM];
  mscale(X * X, F, P->dt, dtF);
  mexp(X, dtF, A);
  mscale(X * X, F, 0.5 * P->dt, hF);
  mexp(X, hF, E2);
  meye(X, I);
  mscale(X * X, E2, 4.0, E2);
  madd(X * X, I, E2, Int);
  madd(X * X, Int, A, Int);
  mscale(X * X, Int, P->dt / 6.0, Int);
  mm(X, X, U, Int, G, B);
  mm(X, X, 1, Int, xdot, c);
}

int orc_synthesize(const lqro_model* m, double* Aout, double* Bout, double* cout,
                   double* Lout, double* Eout, double* Lhout, double* Ehout) {
  return orc_synthesize_x(m, 16, Aout, Bout, cout, Lout, Eout, NULL, Lhout, Ehout);
}

/* jacobi2 (MAT:887-1037): Householder tridiagonalisation + QL iteration
 * (Numerical Recipes, no eigenvalue sort); z = eigenvectors (columns), D =
 * diag(eigenvalues), n x n row-major. */
static void jacobi2(int n, const double* q, double* z, double* D) {
  double d[MXN], e[MXN];
  memcpy(z, q, sizeof(double) * n * n);
  for (int i = 0; i < n; ++i) d[i] = e[i] = 0.0;
  int l, k, j, i, m, iter;
  double scale, hh, h, g, f, s, r = 0.0, p, dd, c, b, absf, absg, pfg;
#define Z(a, bb) z[(a) * n + (bb)]
  for (i = n - 1; i > 0; i--) {
    l = i - 1;
    h = scale = 0.0;
    if (l > 0) {
      for (k = 0; k < i; k++) scale += fabs(Z(i, k));
      if (scale == 0.0) e[i] = Z(i, l);
      else {
        for (k = 0; k < i; k++) { Z(i, k) /= scale; h += Z(i, k) * Z(i, k); }
        f = Z(i, l);
        g = (f >= 0.0 ? -sqrt(h) : sqrt(h));
        e[i] = scale * g;
        h -= f * g;
        Z(i, l) = f - g;
        f = 0.0;
        for (j = 0; j < i; j++) {
          Z(j, i) = Z(i, j) / h;
          g = 0.0;
          for (k = 0; k < j + 1; k++) g += Z(j, k) * Z(i, k);
          for (k = j + 1; k < i; k++) g += Z(k, j) * Z(i, k);
          e[j] = g / h;
          f += e[j] * Z(i, j);
        }
        hh = f / (h + h);
        for (j = 0; j < i; j++) {
          f = Z(i, j);
          e[j] = g = e[j] - hh * f;
          for (k = 0; k < j + 1; k++) Z(j, k) -= (f * e[k] + g * Z(i, k));
        }
      }
    } else {
      e[i] = Z(i, l);
    }
    d[i] = h;
  }
  d[0] = 0.0;
  e[0] = 0.0;
  for (i = 0; i < n; i++) {
    if (d[i] != 0.0) {
      for (j = 0; j < i; j++) {
        g = 0.0;
        for (k = 0; k < i; k++) g += Z(i, k) * Z(k, j);
        for (k = 0; k < i; k++) Z(k, j) -= g * Z(k, i);
      }
    }
    d[i] = Z(i, i);
    Z(i, i) = 1.0;
    for (j = 0; j < i; j++) Z(j, i) = Z(i, j) = 0.0;
  }
  for (i = 1; i < n; i++) e[i - 1] = e[i];
  e[n - 1] = 0.0;
  for (l = 0; l < n; l++) {
    iter = 0;
    do {
      for (m = l; m < n - 1; m++) {
        dd = fabs(d[m]) + fabs(d[m + 1]);
        if (fabs(e[m]) <= DBL_EPSILON * dd) break;
      }
      if (m != l) {
        if (iter++ == 30) break;   /* the reference exits the program here */
        g = (d[l + 1] - d[l]) / (2.0 * e[l]);
        absg = fabs(g);
        r = ((absg > 1.0) ? absg * sqrt(1.0 + (1.0 / absg) * (1.0 / absg)) : sqrt(1.0 + absg * absg));
        g = d[m] - d[l] + e[l] / (g + ((g >= 0.0) ? fabs(r) : -fabs(r)));
        s = c = 1.0;
        p = 0.0;
        for (i = m - 1; i >= l; i--) {
          f = s * e[i];
          b = c * e[i];
          absf = fabs(f);
          absg = fabs(g);
          pfg = (absf > absg ? absf * sqrt(1.0 + (absg / absf) * (absg / absf))
                             : (absg == 0.0 ? 0.0 : absg * sqrt(1.0 + (absf / absg) * (absf / absg))));
          e[i + 1] = (r = pfg);
          if (r == 0.0) { d[i + 1] -= p; e[m] = 0.0; break; }
          s = f / r;
          c = g / r;
          g = d[i + 1] - p;
          r = (d[i] - g) * s + 2.0 * c * b;
          d[i + 1] = g + (p = s * r);
          g = c * r - b;
          for (k = 0; k < n; k++) {
            f = Z(k, i + 1);
            Z(k, i + 1) = s * Z(k, i) + c * f;
            Z(k, i) = c * Z(k, i) - s * f;
          }
        }
        if (r == 0.0 && i >= l) continue;
        d[l] -= p;
        e[l] = g;
        e[m] = 0.0;
      }
    } while (m != l);
  }
#undef Z
  for (i = 0; i < n * n; ++i) D[i] = 0.0;
  for (i = 0; i < n; ++i) D[i * n + i] = d[i];
}

/* pseudoInverse (MAT:450-477) of a square n x n matrix: (Vec Val^+ Vec^T) q^T
 * with jacobi2(q^T q); Val^+ zeroes |eigenvalues| <= sqrt(DBL_EPSILON) */
static void pinv(int n, const double* q, double* out) {
  double qt[MXN * MXN], qtq[MXN * MXN], V[MXN * MXN], D[MXN * MXN], VD[MXN * MXN], Vt[MXN * MXN], VDV[MXN * MXN];
  mt(n, n, q, qt);
  mm(n, n, n, qt, q, qtq);
  jacobi2(n, qtq, V, D);
  for (int i = 0; i < n; ++i) {
    double* v = &D[i * n + i];
    if (fabs(*v) <= sqrt(DBL_EPSILON)) *v = 0.0;
    else *v = 1.0 / *v;
  }
  mm(n, n, n, V, D, VD);
  mt(n, n, V, Vt);
  mm(n, n, n, VD, Vt, VDV);
  mm(n, n, n, VDV, qt, out);
}

void orc_pinv(int n, const double* q, double* out) { pinv(n, q, out); }

/* controlMatrices (LQRO:520-582) for X = 16, or X = 12 (the reduced model of
 * fdyn_x).  Arrays are sized for X = 16 and used with stride X. */
int orc_synthesize_x(const lqro_model* m, int X, double* Aout, double* Bout, double* cout,
                     double* Lout, double* Eout, double* lout, double* Lhout, double* Ehout) {
  enum { XM = 16, U = 4, V = 3 };
  if (X != 16 && X != 12) return -1;
  phys_t P; phys_init(m, &P);
  double nominal = P.gravity * P.mass / 4;   /* LQRO:188 */
  double uGoal[U] = {nominal, nominal, nominal, nominal};
  double xHat[XM] = {0};
  for (int k = 12; k < X; ++k) xHat[k] = nominal;
  double RHat[9]; meye(3, RHat);
  double A[XM * XM], B[XM * U], c[XM];
  linearize(X, &P, xHat, RHat, uGoal, A, B, c);

  double Vm[V * XM] = {0}; Vm[0 * X + 3] = Vm[1 * X + 4] = Vm[2 * X + 5] = 1;
  double Pm[V * XM] = {0}; Pm[0 * X + 0] = Pm[1 * X + 1] = Pm[2 * X + 2] = 1;
  double Qv[9], Qp[9], R[16], I3[9], I4[16];
  meye(3, I3); meye(4, I4);
  mscale(9, I3, m->qv, Qv); mscale(9, I3, m->qp, Qp); mscale(16, I4, m->r, R); /* 5*identity */
  double Qx[XM * XM] = {0};

  double Vt[XM * V], At[XM * XM], Bt[U * XM];
  mt(V, X, Vm, Vt); mt(X, X, A, At); mt(X, U, B, Bt);
  double VtQv[XM * V], VtQvV[XM * XM], nVt[XM * V], nVtQv[XM * V];
  mm(X, V, V, Vt, Qv, VtQv); mm(X, V, X, VtQv, Vm, VtQvV);
  mneg(X * V, Vt, nVt); mm(X, V, V, nVt, Qv, nVtQv);

  double S[XM * XM], T[XM * V];
  memcpy(S, VtQvV, sizeof(double) * X * X);   /* S = ~V*Qv*V */
  memcpy(T, nVtQv, sizeof(double) * X * V);   /* T = -~V*Qv  */
  double AtS[XM * XM], AtSB[XM * U], BtS[U * XM], BtSB[U * U], RB[U * U], Ri[U * U];
  double t1[XM * U], t2[XM * XM], t3[XM * V], AtT[XM * V], BtSA[U * XM], tmp[XM * XM];
  for (int it = 0; it < 300; ++it) {
    /* common: ~A*S*B*!(R + ~B*S*B) with the OLD S */
    mm(X, X, X, At, S, AtS); mm(X, X, U, AtS, B, AtSB);
    mm(U, X, X, Bt, S, BtS); mm(U, X, U, BtS, B, BtSB);
    madd(U * U, R, BtSB, RB); minv(U, RB, Ri);
    mm(X, U, U, AtSB, Ri, t1);
    /* T = -~V*Qv + ~A*T - ~A*S*B*!(..)*~B*T */
    double t1Bt[XM * XM];
    mm(X, U, X, t1, Bt, t1Bt); mm(X, X, V, t1Bt, T, t3);
    mm(X, X, V, At, T, AtT);
    double Tn[XM * V];
    madd(X * V, nVtQv, AtT, Tn); msub(X * V, Tn, t3, Tn);
    /* S = ~V*Qv*V + Qx + ~A*S*A - ~A*S*B*!(..)*(~B*S*A) */
    mm(U, X, X, BtS, A, BtSA);
    mm(X, U, X, t1, BtSA, t2);
    double Sn[XM * XM];
    madd(X * X, VtQvV, Qx, Sn); mm(X, X, X, AtS, A, tmp); madd(X * X, Sn, tmp, Sn);
    msub(X * X, Sn, t2, Sn);
    memcpy(T, Tn, sizeof(double) * X * V); memcpy(S, Sn, sizeof(double) * X * X);
  }
  /* L = -!(R + ~B*S*B)*~B*S*A ; E = -!(R + ~B*S*B)*~B*T  (LQRO:555-556) */
  double L[U * XM], E[U * V], nRi[U * U], tUX[U * XM], tUX2[U * XM];
  mm(U, X, X, Bt, S, BtS); mm(U, X, U, BtS, B, BtSB);
  madd(U * U, R, BtSB, RB); minv(U, RB, Ri); mneg(U * U, Ri, nRi);
  mm(U, U, X, nRi, Bt, tUX); mm(U, X, X, tUX, S, tUX2); mm(U, X, X, tUX2, A, L);
  mm(U, X, V, tUX, T, E);
  if (lout) {
    /* l (LQRO:552, 557), xstar = xHat (Qx*xstar = 0):
     *   a = pseudoInverse(~A - ~A*S*B*!(R+~B*S*B)*~B - I)
     *         * (Qx*xstar - ~A*S*c + ~A*S*B*!(R+~B*S*B)*~B*S*c)
     *   l = -!(R+~B*S*B) * (~B*S*c + ~B*a)                                  */
    double KB[XM * XM], M1[XM * XM], I[XM * XM], Pi[XM * XM], q1[XM], q2[XM], q3[XM], v1[XM], av[XM];
    double KBS[XM * XM], u1[U], u2[U], u3[U];
    mm(X, X, X, At, S, AtS); mm(X, X, U, AtS, B, AtSB);          /* ~A*S*B with the final S */
    mm(U, X, X, Bt, S, BtS); mm(U, X, U, BtS, B, BtSB);
    madd(U * U, R, BtSB, RB); minv(U, RB, Ri);
    mm(X, U, U, AtSB, Ri, t1);                                    /* ~A*S*B*!(..) */
    mm(X, U, X, t1, Bt, KB);                                      /* .. *~B */
    msub(X * X, At, KB, M1); meye(X, I); msub(X * X, M1, I, M1);
    mm(X, X, 1, Qx, xHat, q1);                                    /* Qx*xstar */
    mm(X, X, 1, AtS, c, q2);                                      /* ~A*S*c */
    mm(X, X, X, KB, S, KBS); mm(X, X, 1, KBS, c, q3);             /* ..*~B*S*c */
    msub(X, q1, q2, v1); madd(X, v1, q3, v1);
    pinv(X, M1, Pi);
    mm(X, X, 1, Pi, v1, av);
    mm(U, X, 1, BtS, c, u1); mm(U, X, 1, Bt, av, u2); madd(U, u1, u2, u3);
    mm(U, U, 1, nRi, u3, lout);
  }

  /* position LQR (LQRO:559-581) */
  const double w = m->pos_weight;
  double Pt[XM * V], Lt[XM * U], Et[V * U];
  mt(V, X, Pm, Pt); mt(U, X, L, Lt); mt(U, V, E, Et);
  double Qpt[XM * XM], a1[XM * V], a2[XM * XM], wLt[XM * U], wLtR[XM * U];
  mm(X, V, V, Pt, Qp, a1); mm(X, V, X, a1, Pm, a2);
  mscale(X * U, Lt, w, wLt); mm(X, U, U, wLt, R, wLtR); mm(X, U, X, wLtR, L, tmp);
  madd(X * X, a2, tmp, Qpt);
  double wEt[V * U], wEtR[V * U], Rtl[V * V], Ptl[V * XM];
  mscale(V * U, Et, w, wEt); mm(V, U, U, wEt, R, wEtR);
  mm(V, U, V, wEtR, E, Rtl); mm(V, U, X, wEtR, L, Ptl);
  double Atl[XM * XM], Btl[XM * V], BL[XM * XM];
  mm(X, U, X, B, L, BL); madd(X * X, A, BL, Atl);
  mm(X, U, V, B, E, Btl);

  double St[XM * XM], Tt[XM * V], nPt[XM * V], nPtQp[XM * V];
  memcpy(St, Qpt, sizeof(double) * X * X);
  mneg(X * V, Pt, nPt); mm(X, V, V, nPt, Qp, nPtQp);
  memcpy(Tt, nPtQp, sizeof(double) * X * V);
  double Atlt[XM * XM], Btlt[V * XM], Ptlt[XM * V];
  mt(X, X, Atl, Atlt); mt(X, V, Btl, Btlt); mt(V, X, Ptl, Ptlt);
  double AS[XM * XM], ASB[XM * V], BS[V * XM], BSB[V * V], RR[V * V], RRi[V * V];
  double K1[XM * V], K2[XM * V], BSA[V * XM], PB[V * XM];
  for (int it = 0; it < 300; ++it) {
    mm(X, X, X, Atlt, St, AS); mm(X, X, V, AS, Btl, ASB);
    madd(X * V, Ptlt, ASB, K1);                          /* (~Ptilde + ~At*St*Bt) */
    mm(V, X, X, Btlt, St, BS); mm(V, X, V, BS, Btl, BSB);
    madd(V * V, Rtl, BSB, RR); minv(V, RR, RRi);
    mm(X, V, V, K1, RRi, K2);                            /* (..)*!(..) */
    /* Ttilde = -~P*Qp + ~At*Tt - K2*~Bt*Tt */
    double K2Bt[XM * XM], c3[XM * V], AT[XM * V], Ttn[XM * V];
    mm(X, V, X, K2, Btlt, K2Bt); mm(X, X, V, K2Bt, Tt, c3);
    mm(X, X, V, Atlt, Tt, AT);
    madd(X * V, nPtQp, AT, Ttn); msub(X * V, Ttn, c3, Ttn);
    /* Stilde = Qpt + ~At*St*At - K2*(Ptilde + ~Bt*St*At) */
    double Stn[XM * XM], c4[XM * XM];
    mm(V, X, X, BS, Atl, BSA); madd(V * X, Ptl, BSA, PB);
    mm(X, V, X, K2, PB, c4);
    mm(X, X, X, AS, Atl, tmp); madd(X * X, Qpt, tmp, Stn); msub(X * X, Stn, c4, Stn);
    memcpy(Tt, Ttn, sizeof(double) * X * V); memcpy(St, Stn, sizeof(double) * X * X);
  }
  double Lh[V * XM], Eh[V * V], nRRi[V * V], BtT[V * V];
  mm(V, X, X, Btlt, St, BS); mm(V, X, V, BS, Btl, BSB);
  madd(V * V, Rtl, BSB, RR); minv(V, RR, RRi); mneg(V * V, RRi, nRRi);
  mm(V, X, X, BS, Atl, BSA); madd(V * X, Ptl, BSA, PB);
  mm(V, V, X, nRRi, PB, Lh);
  mm(V, X, V, Btlt, Tt, BtT); mm(V, V, V, nRRi, BtT, Eh);

  if (Aout) memcpy(Aout, A, sizeof(double) * X * X);
  if (Bout) memcpy(Bout, B, sizeof(double) * X * U);
  if (cout) memcpy(cout, c, sizeof(double) * X);
  if (Lout) memcpy(Lout, L, sizeof(double) * U * X);
  if (Eout) memcpy(Eout, E, sizeof(double) * U * V);
  if (Lhout) memcpy(Lhout, Lh, sizeof(double) * V * X);
  if (Ehout) memcpy(Ehout, Eh, sizeof(double) * V * V);
  return 0;
}

/* ------------------------------------------------------------------------ */
/* Sphere + per-agent tables                                                 */
/* ------------------------------------------------------------------------ */
void orc_sphere(int np, double xy_radius, double z_radius, double* s) {
  /* createSpheres, LQRO:735-750 */
  double dlong = M_PI * (3.0 - sqrt(5.0));
  double dz = 2.0 / np;
  double longt = 0;
  double z = 1.0 - dz / 2.0;
  for (int i = 0; i < np; i++) {
    s[i * 3 + 0] = 2 * xy_radius * cos(longt) * sqrt(1 - z * z);
    s[i * 3 + 1] = 2 * xy_radius * sin(longt) * sqrt(1 - z * z);
    s[i * 3 + 2] = 2 * z_radius * z;
    z -= dz;
    longt += dlong;
  }
}

int orc_tables(int X, int U, int H, const double* A, const double* B, const double* L,
               const double* E, double* T, double* NCF) {
  if (X > MXN || U > MXN) return LQRO_E_ARG;
  double F[MXN * MXN], G[MXN * 3], At[MXN * MXN], BL[MXN * MXN], Bt[MXN * 3], t[MXN * 3];
  double C[3 * MXN], nC[3 * MXN], CG[9];
  meye(X, F);
  for (int i = 0; i < X * 3; ++i) G[i] = 0.0;
  for (int i = 0; i < 3 * X; ++i) C[i] = 0.0;
  C[0 * X + 0] = C[1 * X + 1] = C[2 * X + 2] = 1;      /* LQRO:1359-1360 */
  mneg(3 * X, C, nC);
  for (int k = 0; k < H; ++k) {
    /* findFG (LQRO:723-732) */
    mm(X, U, X, B, L, BL); madd(X * X, A, BL, At);
    mm(X, U, 3, B, E, Bt);
    mm(X, X, X, At, F, F);
    mm(X, X, 3, At, G, t); madd(X * 3, t, Bt, G);
    /* createObstacle factors (LQRO:771-773) */
    mm(3, X, 3, C, G, CG);
    minv(3, CG, T + (size_t)k * 9);
    mm(3, X, X, nC, F, NCF + (size_t)k * 3 * X);
    for (int q = 0; q < 9; ++q)
      if (!isfinite(T[(size_t)k * 9 + q])) return LQRO_E_SINGULAR;
  }
  return 0;
}

/* ------------------------------------------------------------------------ */
/* GJK (GJK:86-160, 296-501, 527-736, 770-794, 851-873)                      */
/* ------------------------------------------------------------------------ */
static const int g_card[16] = {0, 1, 1, 2, 1, 2, 2, 3, 1, 2, 2, 3, 2, 3, 3, 4};
static const int g_maxe[16] = {-1, 0, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 3, 3, 3, 3};
static const int g_elts[16][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {1, 0, 0, 0}, {0, 1, 0, 0},
                                  {2, 0, 0, 0}, {0, 2, 0, 0}, {1, 2, 0, 0}, {0, 1, 2, 0},
                                  {3, 0, 0, 0}, {0, 3, 0, 0}, {1, 3, 0, 0}, {0, 1, 3, 0},
                                  {2, 3, 0, 0}, {0, 2, 3, 0}, {1, 2, 3, 0}, {0, 1, 2, 3}};
static const int g_nonelts[16][4] = {{0, 1, 2, 3}, {1, 2, 3, 0}, {0, 2, 3, 0}, {2, 3, 0, 0},
                                     {0, 1, 3, 0}, {1, 3, 0, 0}, {0, 3, 0, 0}, {3, 0, 0, 0},
                                     {0, 1, 2, 0}, {1, 2, 0, 0}, {0, 2, 0, 0}, {2, 0, 0, 0},
                                     {0, 1, 0, 0}, {1, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
static const int g_pred[16][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {2, 1, 0, 0},
                                  {0, 0, 0, 0}, {4, 1, 0, 0}, {4, 2, 0, 0}, {6, 5, 3, 0},
                                  {0, 0, 0, 0}, {8, 1, 0, 0}, {8, 2, 0, 0}, {10, 9, 3, 0},
                                  {8, 4, 0, 0}, {12, 9, 5, 0}, {12, 10, 6, 0}, {14, 13, 11, 7}};
static const int g_succ[16][4] = {{1, 2, 4, 8}, {3, 5, 9, 0}, {3, 6, 10, 0}, {7, 11, 0, 0},
                                  {5, 6, 12, 0}, {7, 13, 0, 0}, {7, 14, 0, 0}, {15, 0, 0, 0},
                                  {9, 10, 12, 0}, {11, 13, 0, 0}, {11, 14, 0, 0}, {15, 0, 0, 0},
                                  {13, 14, 0, 0}, {15, 0, 0, 0}, {15, 0, 0, 0}, {0, 0, 0, 0}};

typedef struct {
  int npts;
  int s2[4];
  double lambdas[4];
  double c1[4][3], c2[4][3];
  double dv[16][4];   /* delta_values (GJK:163) */
  double dp[4][4];    /* dot_products (GJK:164) */
  double dsum[16];    /* delta (GJK:522) */
} gjk_state;

#define GDOT(a, b) ((a)[0] * (b)[0] + (a)[1] * (b)[1] + (a)[2] * (b)[2])

static void gjk_subterms(gjk_state* g) {       /* GJK:527-581 */
  int size = g->npts;
  double csp[4][3];
  for (int i = 0; i < size; i++)
    for (int j = 0; j < 3; j++) csp[i][j] = g->c1[i][j] - g->c2[i][j];
  for (int i = 0; i < size; i++)
    for (int j = i; j < size; j++) g->dp[i][j] = g->dp[j][i] = GDOT(csp[i], csp[j]);
  for (int s = 1; s < 16 && g_maxe[s] < size; s++) {
    if (g_card[s] <= 1) { g->dv[s][g_elts[s][0]] = 1.0; continue; }
    if (g_card[s] == 2) {
      int e0 = g_elts[s][0], e1 = g_elts[s][1];
      g->dv[s][e0] = g->dp[e1][e1] - g->dp[e1][e0];
      g->dv[s][e1] = g->dp[e0][e0] - g->dp[e0][e1];
      continue;
    }
    for (int j = 0; j < g_card[s]; j++) {
      int jelt = g_elts[s][j], jsub = g_pred[s][j];
      double sum = 0;
      for (int i = 0; i < g_card[jsub]; i++) {
        int ielt = g_elts[jsub][i];
        sum += g->dv[jsub][ielt] * (g->dp[ielt][g_elts[jsub][0]] - g->dp[ielt][jelt]);
      }
      g->dv[s][jelt] = sum;
    }
  }
}

static void gjk_reset(gjk_state* g, int subset) {   /* GJK:708-736 */
  for (int j = 0; j < g_card[subset]; j++) {
    int oldpos = g_elts[subset][j];
    if (oldpos != j) {
      g->s2[j] = g->s2[oldpos];
      for (int i = 0; i < 3; i++) { g->c1[j][i] = g->c1[oldpos][i]; g->c2[j][i] = g->c2[oldpos][i]; }
    }
    g->lambdas[j] = g->dv[subset][g_elts[subset][j]] / g->dsum[subset];
  }
  g->npts = g_card[subset];
}

static int gjk_default(gjk_state* g) {        /* GJK:593-657 */
  int s, ok = 0, size = g->npts;
  for (s = 1; s < 16 && g_maxe[s] < size; s++) {
    g->dsum[s] = 0.0; ok = 1;
    for (int j = 0; ok && j < g_card[s]; j++) {
      if (g->dv[s][g_elts[s][j]] > 0.0) g->dsum[s] += g->dv[s][g_elts[s][j]];
      else ok = 0;
    }
    for (int k = 0; ok && k < size - g_card[s]; k++)
      if (g->dv[g_succ[s][k]][g_nonelts[s][k]] > 0) ok = 0;
    if (ok && g->dsum[s] >= 1.0e-20) break;
  }
  if (ok) { gjk_reset(g, s); return 1; }
  return 0;
}

static void gjk_backup(gjk_state* g) {        /* GJK:663-706 */
  int size = g->npts, bests = 0;
  double num[16], den[16];
  for (int s = 1; s < 16 && g_maxe[s] < size; s++) {
    if (g->dsum[s] <= 0.0) continue;
    int i;
    for (i = 0; i < g_card[s]; i++)
      if (g->dv[s][g_elts[s][i]] <= 0.0) break;
    if (i < g_card[s]) continue;
    num[s] = 0.0;
    for (int j = 0; j < g_card[s]; j++)
      for (int k = 0; k < g_card[s]; k++)
        num[s] += (g->dv[s][g_elts[s][j]] * g->dv[s][g_elts[s][k]]) * g->dp[g_elts[s][j]][g_elts[s][k]];
    den[s] = g->dsum[s] * g->dsum[s];
    if ((bests < 1) || (num[s] * den[bests] < num[bests] * den[s])) bests = s;
  }
  gjk_reset(g, bests);
}

static void gjk_point(double pt[3], int len, double (*v)[3], const double* lambdas) {
  for (int d = 0; d < 3; d++) {          /* GJK:851-862 */
    pt[d] = 0;
    for (int i = 0; i < len; i++) pt[d] += v[i][d] * lambdas[i];
  }
}

double orc_gjk(const double vrel[3], int n, const double* pts, double wpt1[3], double wpt2[3],
               int* iters, int* simplex_n, int simplex[4], int* backup) {
  gjk_state g;
  memset(&g, 0, sizeof g);
  int use_default = 1, first_iteration = 1, max_iterations = 1 * n;
  double oldsqrd = 0.0, sqrd = 0.0;
  double disp[3], rdisp[3];
  *iters = 0; *backup = 0;
  g.s2[0] = 0; g.npts = 1; g.lambdas[0] = 1.0;
  for (int d = 0; d < 3; d++) { g.c1[0][d] = vrel[d]; g.c2[0][d] = pts[d]; }
  while (max_iterations-- > 0) {
    if (g.npts == 1) g.lambdas[0] = 1.0;
    else {
      gjk_subterms(&g);
      if (use_default) use_default = gjk_default(&g);
      if (!use_default) { gjk_backup(&g); *backup = 1; }
    }
    gjk_point(wpt1, g.npts, g.c1, g.lambdas);
    gjk_point(wpt2, g.npts, g.c2, g.lambdas);
    for (int d = 0; d < 3; d++) { disp[d] = wpt2[d] - wpt1[d]; rdisp[d] = -disp[d]; }
    sqrd = GDOT(disp, disp);
    if (sqrd < 1.0e-8) goto done;
    double maxv = GDOT(vrel, disp);               /* hill-climb on the 1-vertex ring */
    int minp = 0;
    double minus_minv = GDOT(pts, rdisp);         /* support_simple, GJK:770-794 */
    for (int p = 1; p < n; p++) {
      double thisv = GDOT(pts + 3 * p, rdisp);
      if (thisv > minus_minv) { minus_minv = thisv; minp = p; }
    }
    (*iters)++;
    double g_val = sqrd + maxv + minus_minv;
    if (g_val < 0.0) g_val = 0;
    if (g_val < 1.0e-8) goto done;
    if ((first_iteration || (sqrd < oldsqrd)) && (g.npts <= 3)) {
      g.s2[g.npts] = minp;
      g.lambdas[g.npts] = 0.0;
      for (int d = 0; d < 3; d++) { g.c1[g.npts][d] = vrel[d]; g.c2[g.npts][d] = pts[3 * minp + d]; }
      g.npts++;
      oldsqrd = sqrd;
      first_iteration = 0;
      use_default = 1;
      continue;
    }
    if (use_default) use_default = 0;
    else goto done;
  }
  sqrd = 0.0;
done:
  *simplex_n = g.npts;
  for (int k = 0; k < 4; k++) simplex[k] = k < g.npts ? g.s2[k] : -1;
  return sqrd;
}

/* ------------------------------------------------------------------------ */
/* Hull branch                                                               */
/* ------------------------------------------------------------------------ */
double orc_round6(double v) {
  char buf[64];
  snprintf(buf, sizeof buf, "%g", v);   /* ostream default precision 6 (LQRO:873) */
  return strtod(buf, NULL);
}

typedef struct { int v[3]; double n[3]; double off; int alive; } hface;

typedef struct { long long key; int face; } hedge;

static unsigned hh(long long k, unsigned mask) {
  unsigned long long z = (unsigned long long)k * 0x9E3779B97F4A7C15ull;
  return (unsigned)(z >> 32) & mask;
}

static void face_plane(const double* P, hface* f) {
  const double *a = P + 3 * f->v[0], *b = P + 3 * f->v[1], *c = P + 3 * f->v[2];
  double e1[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
  double e2[3] = {c[0] - a[0], c[1] - a[1], c[2] - a[2]};
  f->n[0] = e1[1] * e2[2] - e1[2] * e2[1];
  f->n[1] = e1[2] * e2[0] - e1[0] * e2[2];
  f->n[2] = e1[0] * e2[1] - e1[1] * e2[0];
  f->off = f->n[0] * a[0] + f->n[1] * a[1] + f->n[2] * a[2];
}
static double face_dist(const double* P, const hface* f, int p) {
  const double* q = P + 3 * p;
  const double* a = P + 3 * f->v[0];
  return f->n[0] * (q[0] - a[0]) + f->n[1] * (q[1] - a[1]) + f->n[2] * (q[2] - a[2]);
}

/* Incremental 3-d hull (beneath-beyond).  Coplanar-within-eps points are not
 * made vertices, as with qconvex's default handling of coplanar points. */
int orc_hull(int n, const double* P, int32_t* out, int cap) {
  if (n < 4) return -1;
  double scale = 0.0;
  for (int i = 0; i < 3 * n; i++) if (fabs(P[i]) > scale) scale = fabs(P[i]);
  const double eps = 1e-13 * (scale + 1.0);
  /* initial simplex: extreme points */
  int i0 = 0;
  for (int i = 1; i < n; i++) if (P[3 * i] < P[3 * i0]) i0 = i;
  int i1 = -1; double best = 0;
  for (int i = 0; i < n; i++) {
    double dx = P[3 * i] - P[3 * i0], dy = P[3 * i + 1] - P[3 * i0 + 1], dz = P[3 * i + 2] - P[3 * i0 + 2];
    double d = dx * dx + dy * dy + dz * dz;
    if (d > best) { best = d; i1 = i; }
  }
  if (i1 < 0) return -2;
  int i2 = -1; best = 0;
  for (int i = 0; i < n; i++) {
    double e1[3] = {P[3 * i1] - P[3 * i0], P[3 * i1 + 1] - P[3 * i0 + 1], P[3 * i1 + 2] - P[3 * i0 + 2]};
    double e2[3] = {P[3 * i] - P[3 * i0], P[3 * i + 1] - P[3 * i0 + 1], P[3 * i + 2] - P[3 * i0 + 2]};
    double cx = e1[1] * e2[2] - e1[2] * e2[1], cy = e1[2] * e2[0] - e1[0] * e2[2], cz = e1[0] * e2[1] - e1[1] * e2[0];
    double d = cx * cx + cy * cy + cz * cz;
    if (d > best) { best = d; i2 = i; }
  }
  if (i2 < 0) return -3;
  hface tmp = {{i0, i1, i2}, {0, 0, 0}, 0, 1};
  face_plane(P, &tmp);
  int i3 = -1; best = 0;
  double nn = sqrt(GDOT(tmp.n, tmp.n));
  for (int i = 0; i < n; i++) {
    double d = fabs(face_dist(P, &tmp, i)) / nn;
    if (d > best) { best = d; i3 = i; }
  }
  if (i3 < 0 || best <= eps) return -4;

  int fcap = 64, fn = 0;
  hface* F = (hface*)malloc(sizeof(hface) * (size_t)fcap);
  unsigned hsize = 1024;
  hedge* E = (hedge*)malloc(sizeof(hedge) * hsize);
  for (unsigned k = 0; k < hsize; k++) E[k].face = -1;
  unsigned hused = 0;
  char* visible = NULL; int viscap = 0;
  int* vis = NULL; int* hor = NULL; int hcap = 0;

#define HKEY(a, b) ((long long)(a) * (long long)n + (long long)(b))
#define EDGE_PUT(a, b, fi)                                                     \
  do {                                                                         \
    if ((hused + 1) * 2 > hsize) {                                             \
      unsigned ns = hsize * 2; hedge* NE = (hedge*)malloc(sizeof(hedge) * ns);  \
      for (unsigned k = 0; k < ns; k++) NE[k].face = -1;                      \
      for (unsigned k = 0; k < hsize; k++)                                     \
        if (E[k].face >= 0) {                                                  \
          unsigned h = hh(E[k].key, ns - 1);                                   \
          while (NE[h].face >= 0) h = (h + 1) & (ns - 1);                      \
          NE[h] = E[k];                                                        \
        }                                                                      \
      free(E); E = NE; hsize = ns;                                             \
    }                                                                          \
    long long key_ = HKEY(a, b); unsigned h_ = hh(key_, hsize - 1);            \
    while (E[h_].face >= 0 && E[h_].key != key_) h_ = (h_ + 1) & (hsize - 1);  \
    if (E[h_].face < 0) hused++;                                               \
    E[h_].key = key_; E[h_].face = (fi);                                       \
  } while (0)

  /* edge lookup; tombstones are face = -2 */
  int rc = 0;
  {
    int tet[4] = {i0, i1, i2, i3};
    int fv[4][3] = {{0, 1, 2}, {0, 3, 1}, {1, 3, 2}, {0, 2, 3}};
    /* orient so the 4th vertex lies below every face */
    for (int f = 0; f < 4; f++) {
      hface h = {{tet[fv[f][0]], tet[fv[f][1]], tet[fv[f][2]]}, {0, 0, 0}, 0, 1};
      face_plane(P, &h);
      int other = tet[6 - fv[f][0] - fv[f][1] - fv[f][2]];
      if (face_dist(P, &h, other) > 0) {
        int t = h.v[1]; h.v[1] = h.v[2]; h.v[2] = t;
        face_plane(P, &h);
      }
      F[fn] = h;
      for (int e = 0; e < 3; e++) EDGE_PUT(h.v[e], h.v[(e + 1) % 3], fn);
      fn++;
    }
  }
  for (int p = 0; p < n; p++) {
    if (p == i0 || p == i1 || p == i2 || p == i3) continue;
    int nv = 0;
    if (viscap < fn) { viscap = fn * 2; visible = (char*)realloc(visible, (size_t)viscap); vis = (int*)realloc(vis, sizeof(int) * (size_t)viscap); }
    for (int f = 0; f < fn; f++) {
      visible[f] = 0;
      if (!F[f].alive) continue;
      /* beyond: d > eps |n|, tested squared as the GPU kernel does */
      const double d = face_dist(P, &F[f], p), nn = GDOT(F[f].n, F[f].n);
      if (d > 0.0 && d * d > eps * eps * nn) { visible[f] = 1; vis[nv++] = f; }
    }
    if (nv == 0) continue;
    /* horizon edges */
    int nh = 0;
    if (hcap < 3 * nv) { hcap = 6 * nv; hor = (int*)realloc(hor, sizeof(int) * 2 * (size_t)hcap); }
    for (int t = 0; t < nv; t++) {
      hface* f = &F[vis[t]];
      for (int e = 0; e < 3; e++) {
        int a = f->v[e], b = f->v[(e + 1) % 3];
        long long key = HKEY(b, a); unsigned h = hh(key, hsize - 1);
        int opp = -1;
        while (E[h].face != -1) {
          if (E[h].face >= 0 && E[h].key == key) { opp = E[h].face; break; }
          h = (h + 1) & (hsize - 1);
        }
        if (opp < 0) { rc = -5; goto out; }
        if (!visible[opp]) { hor[2 * nh] = a; hor[2 * nh + 1] = b; nh++; }
      }
    }
    /* delete visible faces and their edges */
    for (int t = 0; t < nv; t++) {
      hface* f = &F[vis[t]];
      f->alive = 0;
      for (int e = 0; e < 3; e++) {
        long long key = HKEY(f->v[e], f->v[(e + 1) % 3]); unsigned h = hh(key, hsize - 1);
        while (E[h].face != -1) {
          if (E[h].face >= 0 && E[h].key == key) { E[h].face = -2; break; }
          h = (h + 1) & (hsize - 1);
        }
      }
    }
    for (int t = 0; t < nh; t++) {
      if (fn == fcap) { fcap *= 2; F = (hface*)realloc(F, sizeof(hface) * (size_t)fcap); }
      hface h = {{hor[2 * t], hor[2 * t + 1], p}, {0, 0, 0}, 0, 1};
      face_plane(P, &h);
      F[fn] = h;
      for (int e = 0; e < 3; e++) EDGE_PUT(h.v[e], h.v[(e + 1) % 3], fn);
      fn++;
    }
  }
  {
    int cnt = 0;
    for (int f = 0; f < fn; f++) {
      if (!F[f].alive) continue;
      if (cnt < cap) { out[3 * cnt] = F[f].v[0]; out[3 * cnt + 1] = F[f].v[1]; out[3 * cnt + 2] = F[f].v[2]; }
      cnt++;
    }
    rc = cnt;
  }
out:
  free(F); free(E); free(visible); free(vis); free(hor);
  return rc;
#undef HKEY
#undef EDGE_PUT
}

/* canonical facet order: (lowest vertex, then the other two ascending) */
static int tri_cmp(const void* a, const void* b) {
  const int32_t* x = (const int32_t*)a; const int32_t* y = (const int32_t*)b;
  int32_t kx[3] = {x[0], x[1] < x[2] ? x[1] : x[2], x[1] < x[2] ? x[2] : x[1]};
  int32_t ky[3] = {y[0], y[1] < y[2] ? y[1] : y[2], y[1] < y[2] ? y[2] : y[1]};
  for (int k = 0; k < 3; k++) if (kx[k] != ky[k]) return kx[k] < ky[k] ? -1 : 1;
  return 0;
}

/* rotate an oriented triangle so its smallest index comes first */
static void tri_canon(int32_t* t) {
  while (!(t[0] < t[1] && t[0] < t[2])) { int32_t a = t[0]; t[0] = t[1]; t[1] = t[2]; t[2] = a; }
}

int orc_hull_branch(int n, const double* pts_full, const double vrel[3], double* dist,
                    double normal[3], int facet[3]) {
  double* rp = (double*)malloc(sizeof(double) * 3 * (size_t)n);
  for (int i = 0; i < 3 * n; i++) rp[i] = orc_round6(pts_full[i]);
  int cap = 4 * n + 16;
  int32_t* fc = (int32_t*)malloc(sizeof(int32_t) * 3 * (size_t)cap);
  int nf = orc_hull(n, rp, fc, cap);
  if (nf <= 0) { free(rp); free(fc); return nf; }
  for (int f = 0; f < nf; f++) tri_canon(fc + 3 * f);
  qsort(fc, (size_t)nf, sizeof(int32_t) * 3, tri_cmp);
  for (int f = 0; f < nf; f++) {
    const int32_t* t = fc + 3 * f;
    const double *a = rp + 3 * t[0], *b = rp + 3 * t[1], *c = rp + 3 * t[2];
    double e1[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
    double e2[3] = {c[0] - a[0], c[1] - a[1], c[2] - a[2]};
    double nv[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
    double len = sqrt(nv[0] * nv[0] + nv[1] * nv[1] + nv[2] * nv[2]);
    nv[0] /= len; nv[1] /= len; nv[2] /= len;
    const double* p0 = pts_full + 3 * t[0];
    double d = fabs(nv[0] * (vrel[0] - p0[0]) + nv[1] * (vrel[1] - p0[1]) + nv[2] * (vrel[2] - p0[2]));
    if (f == 0 || d < *dist) {
      *dist = d;
      normal[0] = nv[0]; normal[1] = nv[1]; normal[2] = nv[2];
      facet[0] = t[0];
      facet[1] = t[1] < t[2] ? t[1] : t[2];
      facet[2] = t[1] < t[2] ? t[2] : t[1];
    }
  }
  free(rp); free(fc);
  return nf;
}

/* The reference's own selection rule (convexHull, LQRO:867-969) over
 * Qhull's output (lqro_qhull.c): facets in Qhull's order, each measured from
 * its FIRST Fv vertex at full precision (LQRO:934-937), strict '<'
 * (LQRO:955-967); facet 0 never writes `normal` (LQRO:956-958): *stale = 1
 * then, and the caller keeps the loop-carried normalVector.  round16 = 1
 * reads the planes back as qconvex prints them (%.16g, LQRO:895-899).
 * *qstatus: lqro_qhull.h QHO_* bits (non-zero: Qhull would have merged
 * facets; the hull was built on merge-free).  Returns the facet count or
 * <= 0 on failure. */
static int g_hull_rule = 0, g_round16 = 0;
#define ORC_QH_MERGE_WIN 0x10000   /* orc_hull_branch_ref's *qstatus: LQRO_REC_QHMERGE_WIN */
#define ORC_QH_MERGE_WIN_LOOSE 0x20000   /* diagnostics: round 5's looser test (1e-9 (|coord|max + 1)) */
#define ORC_QH_MERGE_K 1024.0      /* the suspect test's reach, in units of qh DISTround */
static long long g_hull_ns = 0, g_hull_count = 0;

/* time spent in the hull branch and inside-hull pairs since the last reset */
void orc_hull_time(double* seconds, long long* count, int reset) {
  *seconds = 1e-9 * (double)__atomic_load_n(&g_hull_ns, __ATOMIC_RELAXED);
  *count = __atomic_load_n(&g_hull_count, __ATOMIC_RELAXED);
  if (reset) {
    __atomic_store_n(&g_hull_ns, 0LL, __ATOMIC_RELAXED);
    __atomic_store_n(&g_hull_count, 0LL, __ATOMIC_RELAXED);
  }
}
static double g_carry[3] = {0.0, 0.0, 0.0};

void orc_set_hull_rule(int rule, int round16) { g_hull_rule = rule; g_round16 = round16; }
void orc_set_carry_normal(const double* n) { g_carry[0] = n[0]; g_carry[1] = n[1]; g_carry[2] = n[2]; }
void orc_get_carry_normal(double* n) { n[0] = g_carry[0]; n[1] = g_carry[1]; n[2] = g_carry[2]; }

static double g16(double v) {
  char b[64];
  snprintf(b, sizeof b, "%.16g", v);
  return strtod(b, NULL);
}

int orc_hull_branch_ref(int n, const double* pts_full, const double vrel[3], double* dist,
                        double normal[3], int facet[3], int* stale, int* qstatus) {
  double* rp = (double*)malloc(sizeof(double) * 3 * (size_t)n);
  for (int i = 0; i < 3 * n; i++) rp[i] = orc_round6(pts_full[i]);      /* LQRO:871-873 */
  orc_qhull_out o;
  const int nf = orc_qhull_ex(rp, n, &o, 1);
  *qstatus = o.status;
  *stale = 0;
  if (nf <= 0) { orc_qhull_free(&o); free(rp); return nf <= 0 ? -1 : nf; }
  int best = 0;
  double d = 0.0;
  for (int f = 0; f < nf; f++) {
    double pl[3];
    for (int k = 0; k < 3; k++) pl[k] = g_round16 ? g16(o.plane[4 * f + k]) : o.plane[4 * f + k];
    const double* P = pts_full + 3 * (size_t)o.fv[3 * f];              /* first Fv vertex */
    const double t = fabs(pl[0] * (vrel[0] - P[0]) + pl[1] * (vrel[1] - P[1]) + pl[2] * (vrel[2] - P[2]));
    if (f == 0 || t < d) {
      d = t;
      best = f;
      if (f > 0) { normal[0] = pl[0]; normal[1] = pl[1]; normal[2] = pl[2]; }
    }
  }
  *dist = d;
  *stale = best == 0;
  for (int k = 0; k < 3; k++) facet[k] = o.fv[3 * best + k];
  /* LQRO_REC_QHMERGE_WIN (reported as *qstatus bit ORC_QH_MERGE_WIN): Qhull's
   * merge tests fired in this build, and a facet that can decide the rule —
   * one within 1e-6 of the winning distance, or facet 0 (the list head, whose
   * merge would change which facet keeps the loop-carried normal) — has
   * another hull vertex within ORC_QH_MERGE_K x qh DISTround of its plane:
   * qconvex's pre-merge (centrum radius 2 DISTround for C-0, coplanar
   * horizon 2 DISTround, qh_checkzero 2 DISTround) may have joined it with a
   * neighbour, so the reference's winner may be a merged facet (LQRO:925-967).
   * The GPU's q3_merge_suspect / qh_merge_suspect, same arithmetic.  Round 5's
   * reach of 1e-9 (|coord|max + 1), ~1e6 x DISTround, also flagged hulls
   * whose qconvex merge is far from the winner (C5: 35 of 2048 rows' pairs,
   * every one checked against live Qhull simplicial at the winner); it is
   * kept as a diagnostic bit. */
  if (o.status) {
    double maxabs = 0.0;
    for (int i = 0; i < 3 * n; i++) maxabs = fabs(rp[i]) > maxabs ? fabs(rp[i]) : maxabs;
    const double Tl = -1e-9 * (maxabs + 1.0);
    const double T = -ORC_QH_MERGE_K * o.distround;
    int sus = 0, lsus = 0;
    for (int f = 0; f < nf && !(sus && lsus); f++) {
      const double* q = o.plane + 4 * f;
      const double* P = pts_full + 3 * (size_t)o.fv[3 * f];
      const int near = fabs(q[0] * (vrel[0] - P[0]) + q[1] * (vrel[1] - P[1]) + q[2] * (vrel[2] - P[2])) <= d + 1e-6;
      if (!near && f != 0) continue;
      for (int g = 0; g < 3 * nf; g++) {
        const int id = o.fv[g];
        if (id == o.fv[3 * f] || id == o.fv[3 * f + 1] || id == o.fv[3 * f + 2]) continue;
        const double* p = rp + 3 * (size_t)id;
        const double dv = q[3] + p[0] * q[0] + p[1] * q[1] + p[2] * q[2];
        if (dv >= T) sus = 1;
        if (near && dv >= Tl) lsus = 1;
      }
    }
    if (sus) *qstatus |= ORC_QH_MERGE_WIN;
    if (lsus) *qstatus |= ORC_QH_MERGE_WIN_LOOSE;
  }
  orc_qhull_free(&o);
  free(rp);
  return nf;
}

/* ------------------------------------------------------------------------ */
/* Per pair                                                                   */
/* ------------------------------------------------------------------------ */
static uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

int orc_pair(int X, int H, int NP, int min_reach, double vmax_reach, const double* T,
             const double* NCF, const double* S, const double* xi, const double* xj, int i,
             int j, lqro_pair_record* rec, int32_t* reach_idx, double* reach_pts) {
  if (X > MXN) return LQRO_E_ARG;
  double* pts = reach_pts;
  int own = 0;
  if (!pts) { pts = (double*)malloc(sizeof(double) * 3 * (size_t)H * (size_t)NP); own = 1; }
  double d[MXN];
  for (int c = 0; c < X; c++) d[c] = xi[c] - xj[c];              /* (xInit1-xInit2) */
  const double xc = xi[3] - xj[3], yc = xi[4] - xj[4], zc = xi[5] - xj[5]; /* LQRO:794-796 */
  const double r2 = vmax_reach * vmax_reach;                     /* pow(maxSpeed,2) */
  int n = 0;
  uint64_t hsh = 0;
  for (int k = 0; k < H; k++) {
    const double* nc = NCF + (size_t)k * 3 * X;
    const double* Tk = T + (size_t)k * 9;
    double tr[3];
    for (int r = 0; r < 3; r++) {                                 /* Translate, LQRO:773 */
      double temp = 0.0;
      for (int c = 0; c < X; c++) temp += nc[r * X + c] * d[c];
      tr[r] = temp;
    }
    for (int p = 0; p < NP; p++) {                                /* LQRO:775-776 */
      double u[3] = {S[3 * p] + tr[0], S[3 * p + 1] + tr[1], S[3 * p + 2] + tr[2]};
      double pt[3];
      for (int r = 0; r < 3; r++) {
        double temp = 0.0;
        for (int c = 0; c < 3; c++) temp += Tk[r * 3 + c] * u[c];
        pt[r] = temp;
      }
      /* findReachableObstacle, LQRO:798-801 */
      double a = pt[0] - xc, b = pt[1] - yc, cc = pt[2] - zc;
      if ((a * a) / r2 + (b * b) / r2 + (cc * cc) / r2 < 1.0) {
        if (reach_idx) reach_idx[n] = k * NP + p;
        hsh += mix64((uint64_t)(k * NP + p));
        pts[3 * n] = pt[0]; pts[3 * n + 1] = pt[1]; pts[3 * n + 2] = pt[2];
        n++;
      }
    }
  }
  memset(rec, 0, sizeof *rec);
  rec->i = i; rec->j = j; rec->n_reach = n; rec->reach_hash = hsh;
  rec->facet[0] = rec->facet[1] = rec->facet[2] = -1;
  for (int k = 0; k < 4; k++) rec->simplex[k] = -1;
  if (n > min_reach) {                                            /* LQRO:1409 */
    double vrel[3] = {xc, yc, zc};
    double w1[3], w2[3];
    int iters, sn, backup;
    double sq = orc_gjk(vrel, n, pts, w1, w2, &iters, &sn, rec->simplex, &backup);
    double distance = sqrt(sq);                                   /* LQRO:843 */
    double normal[3] = {(w1[0] - w2[0]) / distance, (w1[1] - w2[1]) / distance,
                        (w1[2] - w2[2]) / distance};              /* LQRO:850-852 */
    int inside = (distance < 0.0001 && distance > -1 * 0.0001);   /* LQRO:858-861 */
    rec->flags = LQRO_REC_PLANE | (inside ? LQRO_REC_INSIDE : 0) | (backup ? LQRO_REC_BACKUP : 0);
    rec->gjk_iters = iters; rec->simplex_n = sn;
    for (int k = 0; k < 3; k++) { rec->wpt_vrel[k] = w1[k]; rec->wpt_hull[k] = w2[k]; }
    int stale = 0;
    struct timespec h0, h1;
    if (inside) clock_gettime(CLOCK_MONOTONIC, &h0);
    if (inside && g_hull_rule) {                                  /* LQRO:1411-1412 */
      int qst = 0;
      int nf = orc_hull_branch_ref(n, pts, vrel, &distance, normal, rec->facet, &stale, &qst);
      rec->n_facets = nf;
      if (nf > 0) rec->flags |= LQRO_REC_HULL; else rec->flags |= LQRO_REC_HULLFAIL;
      if (qst) rec->flags |= LQRO_REC_QHMERGE;
      if (qst & ORC_QH_MERGE_WIN) rec->flags |= LQRO_REC_QHMERGE_WIN;
      if (stale) {   /* normalVector keeps the previous pair's value: resolved by the row loop */
        rec->flags |= LQRO_REC_STALE;
        normal[0] = normal[1] = normal[2] = 0.0;
      }
    } else if (inside) {
      int nf = orc_hull_branch(n, pts, vrel, &distance, normal, rec->facet);
      rec->n_facets = nf;
      if (nf > 0) rec->flags |= LQRO_REC_HULL; else rec->flags |= LQRO_REC_HULLFAIL;
    }
    if (inside) {   /* the hull branch's cost (the CPU baseline reports it apart) */
      clock_gettime(CLOCK_MONOTONIC, &h1);
      __atomic_add_fetch(&g_hull_ns, (long long)(h1.tv_sec - h0.tv_sec) * 1000000000LL + (h1.tv_nsec - h0.tv_nsec),
                         __ATOMIC_RELAXED);
      __atomic_add_fetch(&g_hull_count, 1LL, __ATOMIC_RELAXED);
    }
    rec->dist = distance;
    for (int k = 0; k < 3; k++) rec->normal[k] = normal[k];
    distance *= 0.5;                                              /* LQRO:1416 */
    double mult = inside ? 1.0 : -1.0;                            /* LQRO:1212-1215 */
    rec->plane_normal[0] = (float)normal[0]; rec->plane_normal[1] = (float)normal[1];
    rec->plane_normal[2] = (float)normal[2];
    rec->plane_point[0] = (float)(xi[3] + mult * distance * normal[0]);
    rec->plane_point[1] = (float)(xi[4] + mult * distance * normal[1]);
    rec->plane_point[2] = (float)(xi[5] + mult * distance * normal[2]);
  }
  if (own) free(pts);
  return 0;
}

/* ------------------------------------------------------------------------ */
/* RVO2-3D LP in fp32 (LQRO:971-1234, Vector3.h)                              */
/* ------------------------------------------------------------------------ */
typedef struct { float x, y, z; } v3;
typedef struct { v3 point, normal; } plane_t;
typedef struct { v3 point, direction; } line_t;

static v3 V(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static float vdot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static v3 vadd(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static v3 vsub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static v3 vmul(v3 a, float s) { return V(a.x * s, a.y * s, a.z * s); }   /* Vector3*float */
static v3 smul(float s, v3 a) { return V(s * a.x, s * a.y, s * a.z); }   /* float*Vector3 */
static v3 vcross(v3 a, v3 b) {
  return V(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static float vabsSq(v3 a) { return vdot(a, a); }
static v3 vnormalize(v3 a) {
  float l = sqrtf(vdot(a, a));
  const float invS = 1.0f / l;
  return V(a.x * invS, a.y * invS, a.z * invS);
}
static float sqrf(float s) { return s * s; }
static float fmaxs(float a, float b) { return (a < b) ? b : a; }  /* std::max */
static float fmins(float a, float b) { return (b < a) ? b : a; }  /* std::min */

#define RVO_EPSILON 0.00001f

/* the length of the LP's sequential chain (linearProgram1 calls plus
 * violated planes met by the scans of linearProgram2-4) since the last
 * orc_lp_chain: test instrumentation only, it does not change any result */
static __thread long long g_lp_chain;

static int lp1(const plane_t* planes, int planeNo, const line_t* line, float radius, v3 optVelocity,
               int directionOpt, v3* result) {
  g_lp_chain++;
  const float dotProduct = vdot(line->point, line->direction);
  const float discriminant = sqrf(dotProduct) + sqrf(radius) - vabsSq(line->point);
  if (discriminant < 0.0f) return 0;
  const float sqrtDiscriminant = sqrtf(discriminant);
  float tLeft = -dotProduct - sqrtDiscriminant;
  float tRight = -dotProduct + sqrtDiscriminant;
  for (int i = 0; i < planeNo; ++i) {
    const float numerator = vdot(vsub(planes[i].point, line->point), planes[i].normal);
    const float denominator = vdot(line->direction, planes[i].normal);
    if (sqrf(denominator) <= RVO_EPSILON) {
      if (numerator > 0.0f) return 0;
      else continue;
    }
    const float t = numerator / denominator;
    if (denominator >= 0.0f) tLeft = fmaxs(tLeft, t);
    else tRight = fmins(tRight, t);
    if (tLeft > tRight) return 0;
  }
  if (directionOpt) {
    if (vdot(optVelocity, line->direction) > 0.0f) *result = vadd(line->point, smul(tRight, line->direction));
    else *result = vadd(line->point, smul(tLeft, line->direction));
  } else {
    const float t = vdot(line->direction, vsub(optVelocity, line->point));
    if (t < tLeft) *result = vadd(line->point, smul(tLeft, line->direction));
    else if (t > tRight) *result = vadd(line->point, smul(tRight, line->direction));
    else *result = vadd(line->point, smul(t, line->direction));
  }
  return 1;
}

static int lp2(const plane_t* planes, int planeNo, float radius, v3 optVelocity, int directionOpt,
               v3* result) {
  const float planeDist = vdot(planes[planeNo].point, planes[planeNo].normal);
  const float planeDistSq = sqrf(planeDist);
  const float radiusSq = sqrf(radius);
  if (planeDistSq > radiusSq) return 0;
  const float planeRadiusSq = radiusSq - planeDistSq;
  const v3 planeCenter = smul(planeDist, planes[planeNo].normal);
  if (directionOpt) {
    const v3 planeOptVelocity =
        vsub(optVelocity, smul(vdot(optVelocity, planes[planeNo].normal), planes[planeNo].normal));
    const float planeOptVelocityLengthSq = vabsSq(planeOptVelocity);
    if (planeOptVelocityLengthSq <= RVO_EPSILON) *result = planeCenter;
    else *result = vadd(planeCenter, smul(sqrtf(planeRadiusSq / planeOptVelocityLengthSq), planeOptVelocity));
  } else {
    *result = vadd(optVelocity, smul(vdot(vsub(planes[planeNo].point, optVelocity), planes[planeNo].normal),
                                     planes[planeNo].normal));
    if (vabsSq(*result) > radiusSq) {
      const v3 planeResult = vsub(*result, planeCenter);
      const float planeResultLengthSq = vabsSq(planeResult);
      *result = vadd(planeCenter, smul(sqrtf(planeRadiusSq / planeResultLengthSq), planeResult));
    }
  }
  for (int i = 0; i < planeNo; ++i) {
    if (vdot(planes[i].normal, vsub(planes[i].point, *result)) > 0.0f) {
      g_lp_chain++;
      v3 crossProduct = vcross(planes[i].normal, planes[planeNo].normal);
      if (vabsSq(crossProduct) <= RVO_EPSILON) return 0;
      line_t line;
      line.direction = vnormalize(crossProduct);
      const v3 lineNormal = vcross(line.direction, planes[planeNo].normal);
      line.point = vadd(planes[planeNo].point,
                        smul(vdot(vsub(planes[i].point, planes[planeNo].point), planes[i].normal) /
                                 vdot(lineNormal, planes[i].normal),
                             lineNormal));
      if (!lp1(planes, i, &line, radius, optVelocity, directionOpt, result)) return 0;
    }
  }
  return 1;
}

static int lp3(const plane_t* planes, int m, double radius, v3 optVelocity, int directionOpt,
               v3* result) {
  if (directionOpt) *result = vmul(optVelocity, (float)radius);
  else if (vabsSq(optVelocity) > sqrf((float)radius)) *result = vmul(vnormalize(optVelocity), (float)radius);
  else *result = optVelocity;
  for (int i = 0; i < m; ++i) {
    if (vdot(planes[i].normal, vsub(planes[i].point, *result)) > 0.0f) {
      g_lp_chain++;
      const v3 tempResult = *result;
      if (!lp2(planes, i, (float)radius, optVelocity, directionOpt, result)) {
        *result = tempResult;
        return i;
      }
    }
  }
  return m;
}

static void lp4(const plane_t* planes, int m, int beginPlane, float radius, v3* result,
                plane_t* scratch) {
  float distance = 0.0f;
  for (int i = beginPlane; i < m; ++i) {
    if (vdot(planes[i].normal, vsub(planes[i].point, *result)) > distance) {
      g_lp_chain++;
      int np = 0;
      for (int j = 0; j < i; ++j) {
        plane_t plane;
        const v3 crossProduct = vcross(planes[j].normal, planes[i].normal);
        if (vabsSq(crossProduct) <= RVO_EPSILON) {
          if (vdot(planes[i].normal, planes[j].normal) > 0.0f) continue;
          else plane.point = smul(0.5f, vadd(planes[i].point, planes[j].point));
        } else {
          const v3 lineNormal = vcross(crossProduct, planes[i].normal);
          plane.point = vadd(planes[i].point,
                             smul(vdot(vsub(planes[j].point, planes[i].point), planes[j].normal) /
                                      vdot(lineNormal, planes[j].normal),
                                  lineNormal));
        }
        plane.normal = vnormalize(vsub(planes[j].normal, planes[i].normal));
        scratch[np++] = plane;
      }
      const v3 tempResult = *result;
      if (lp3(scratch, np, radius, planes[i].normal, 1, result) < np) *result = tempResult;
      distance = vdot(planes[i].normal, vsub(planes[i].point, *result));
    }
  }
}

void orc_newv(int m, const float* pl, const double* vgoal, double vmax_lp, double* newv) {
  plane_t* planes = (plane_t*)malloc(sizeof(plane_t) * (size_t)(m > 0 ? m : 1));
  plane_t* scratch = (plane_t*)malloc(sizeof(plane_t) * (size_t)(m > 0 ? m : 1));
  for (int k = 0; k < m; k++) {
    planes[k].point = V(pl[6 * k], pl[6 * k + 1], pl[6 * k + 2]);
    planes[k].normal = V(pl[6 * k + 3], pl[6 * k + 4], pl[6 * k + 5]);
  }
  const double maxSpeed_ = vmax_lp;                              /* LQRO:1224 */
  v3 pref = V((float)vgoal[0], (float)vgoal[1], (float)vgoal[2]);
  v3 nv = V(0.0f, 0.0f, 0.0f);
  int planeFail = lp3(planes, m, maxSpeed_, pref, 0, &nv);       /* LQRO:1228 */
  if (planeFail < m) lp4(planes, m, planeFail, (float)maxSpeed_, &nv, scratch);
  newv[0] = nv.x; newv[1] = nv.y; newv[2] = nv.z;
  free(planes); free(scratch);
}

/* linearProgram4's share of the sequential chain of calculateNewV for one
 * plane list (0 when linearProgram3 succeeds): ranks the hardest LPs for
 * tests/golden/make_golden_lp_rows.py */
long long orc_lp_chain(int m, const float* pl, const double* vgoal, double vmax_lp) {
  double nv[3];
  long long c0;
  plane_t* planes = (plane_t*)malloc(sizeof(plane_t) * (size_t)(m > 0 ? m : 1));
  for (int k = 0; k < m; k++) {
    planes[k].point = V(pl[6 * k], pl[6 * k + 1], pl[6 * k + 2]);
    planes[k].normal = V(pl[6 * k + 3], pl[6 * k + 4], pl[6 * k + 5]);
  }
  v3 pref = V((float)vgoal[0], (float)vgoal[1], (float)vgoal[2]);
  v3 r = V(0.0f, 0.0f, 0.0f);
  const int fail = lp3(planes, m, vmax_lp, pref, 0, &r);
  free(planes);
  if (fail >= m) return 0;
  c0 = g_lp_chain;
  orc_newv(m, pl, vgoal, vmax_lp, nv);
  return g_lp_chain - c0;
}

/* operator! on a 3x3 / 4x4 matrix (MAT:603-671), for the tests */
void orc_inverse3(const double* in, double* out) { minv(3, in, out); }
void orc_inverse4(const double* in, double* out) { minv(4, in, out); }

/* ------------------------------------------------------------------------ */
/* Whole step                                                                */
/* ------------------------------------------------------------------------ */
/* Opt-in neighbour culling (SURVEY §8f next #3, RVO2 computeNeighbors /
 * insertAgentNeighbor, AGT:74-81,153-174): agent i keeps the max_nbr agents
 * j != i with the smallest d2 = |p_i - p_j|^2 < nbr_dist^2, ties to the lower
 * j (RVO2 keeps the earlier-visited one).  Only their pairs are computed, and
 * the LP sees their planes in j order.  0 neighbours = all pairs (the
 * reference's loop). */
static double g_nbr_r2 = 0.0;
static int g_nbr_k = 0;

void orc_set_neighbors(double nbr_dist, int max_nbr) {
  g_nbr_r2 = nbr_dist * nbr_dist;
  g_nbr_k = max_nbr;
}

static double nbr_d2(const double* x, int X, int i, int j) {
  const double dx = x[(size_t)i * X] - x[(size_t)j * X];
  const double dy = x[(size_t)i * X + 1] - x[(size_t)j * X + 1];
  const double dz = x[(size_t)i * X + 2] - x[(size_t)j * X + 2];
  return dx * dx + dy * dy + dz * dz;
}

/* sel[j] = 1 for agent i's neighbours (RVO2's sorted insertion, restated) */
void orc_neighbors(int N, int X, const double* x, int i, double r2, int k, unsigned char* sel) {
  double* kd = (double*)malloc(sizeof(double) * (size_t)(k > 0 ? k : 1));
  int* kj = (int*)malloc(sizeof(int) * (size_t)(k > 0 ? k : 1));
  int n = 0;
  double range = r2;
  for (int j = 0; j < N; ++j) {
    sel[j] = 0;
    if (j == i) continue;
    const double d2 = nbr_d2(x, X, i, j);
    if (!(d2 < range)) continue;
    if (n < k) n++;
    int p = n - 1;
    while (p != 0 && d2 < kd[p - 1]) { kd[p] = kd[p - 1]; kj[p] = kj[p - 1]; --p; }
    kd[p] = d2; kj[p] = j;
    if (n == k) range = kd[n - 1];
  }
  for (int q = 0; q < n; ++q) sel[kj[q]] = 1;
  free(kd); free(kj);
}

/* The gains of the reference-faithful mode (orc_step_faithful): A, B shared,
 * L, E one block or per agent. */
typedef struct {
  const double *A, *B, *L, *E;
} faith_t;

/* Qhull-order rule: the loop-carried normalVector (LQRO:1385) across the
 * pairs of a row is resolved in step_rows; a row whose first eligible pairs
 * are stale waits for the previous row's last normal (rows run on several
 * threads): its planes are kept and resolve_rows finishes it in row order. */
typedef struct {
  int kind;            /* 0: no eligible pair; 1: `last` is the row's last normal; */
                       /* 2: every eligible pair is a leading stale pair          */
  double last[3];
  int m, nlead;
  float* planes;       /* m x 6, kept when nlead > 0 */
  int* lead_plane;     /* plane index of each leading stale pair */
  int* lead_rec;       /* its record index */
  double* lead_dist;   /* its 0.5 * dist */
} rowstate_t;

static void stale_plane(const double* xi, double half_dist, const double* n, float* pp, float* pn) {
  const double mult = 1.0;                                        /* inside, LQRO:1212-1213 */
  for (int k = 0; k < 3; k++) {
    pn[k] = (float)n[k];
    pp[k] = (float)(xi[3 + k] + mult * half_dist * n[k]);
  }
}

static int step_rows(int N, int X, int H, int NP, int min_reach, double vmax_reach, double vmax_lp,
                     int per_agent, const double* T, const double* NCF, const double* S,
                     const double* x, const double* vgoal, int r0, int r1, double* newv,
                     lqro_pair_record* recs, const faith_t* fa, rowstate_t* rs) {
  unsigned char* sel = (unsigned char*)malloc((size_t)N);
  double* pts = (double*)malloc(sizeof(double) * 3 * (size_t)H * (size_t)NP);
  float* planes = (float*)malloc(sizeof(float) * 6 * (size_t)(N > 1 ? N - 1 : 1));
  double* Tf = fa ? (double*)malloc(sizeof(double) * 9 * (size_t)H) : NULL;
  double* Nf = fa ? (double*)malloc(sizeof(double) * 3 * (size_t)X * (size_t)H) : NULL;
  lqro_pair_record rec;
  int rc = 0;
  for (int i = r0; i < r1; ++i) {
    const double* Ti = per_agent ? T + (size_t)i * H * 9 : T;
    const double* Ni = per_agent ? NCF + (size_t)i * H * 3 * X : NCF;
    if (fa) { Ti = Tf; Ni = Nf; }
    int m = 0;
    int have = 0, nlead = 0;
    double cur[3] = {0.0, 0.0, 0.0};
    int* lead_plane = NULL;
    int* lead_rec = NULL;
    double* lead_dist = NULL;
    if (g_nbr_k > 0) orc_neighbors(N, X, x, i, g_nbr_r2, g_nbr_k, sel);
    for (int j = 0; j < N; ++j) {
      if (j == i) continue;
      if (g_nbr_k > 0 && !sel[j]) {   /* culled: no pair, no plane */
        if (recs) {
          lqro_pair_record* r = &recs[(size_t)(i - r0) * (N - 1) + (j < i ? j : j - 1)];
          memset(r, 0, sizeof *r);
          r->i = i; r->j = j; r->n_reach = -1;
        }
        continue;
      }
      if (fa) {
        /* per pair, as LQRO:1401-1406: F = I, G = 0, then H x (findFG +
         * createObstacle's Transform = !(C*G), -C*F) — orc_tables is that
         * recursion (Atilde, Btilde recomputed every k, LQRO:723-732) */
        const double* Li = fa->L + (per_agent ? (size_t)i * 4 * X : 0);
        const double* Ei = fa->E + (per_agent ? (size_t)i * 4 * 3 : 0);
        rc = orc_tables(X, 4, H, fa->A, fa->B, Li, Ei, Tf, Nf);
        if (rc) goto out;
      }
      rc = orc_pair(X, H, NP, min_reach, vmax_reach, Ti, Ni, S, x + (size_t)i * X,
                    x + (size_t)j * X, i, j, &rec, NULL, pts);
      if (rc) goto out;
      if (fa && (rec.flags & LQRO_REC_PLANE) && !(rec.flags & LQRO_REC_INSIDE)) {
        /* run_gjk (LQRO:1414) repeats pointInHull's GJK (LQRO:1410) */
        const double* xi = x + (size_t)i * X;
        const double* xj = x + (size_t)j * X;
        double vrel[3] = {xi[3] - xj[3], xi[4] - xj[4], xi[5] - xj[5]}, w1[3], w2[3];
        int it2, sn2, bk2, simp[4];
        volatile double sq2 = orc_gjk(vrel, rec.n_reach, pts, w1, w2, &it2, &sn2, simp, &bk2);
        (void)sq2;
      }
      if (rs && (rec.flags & LQRO_REC_PLANE)) {
        if (rec.flags & LQRO_REC_STALE) {
          if (have) {
            for (int k = 0; k < 3; k++) rec.normal[k] = cur[k];
            stale_plane(x + (size_t)i * X, 0.5 * rec.dist, cur, rec.plane_point, rec.plane_normal);
          } else {
            if (!lead_plane) {
              lead_plane = (int*)malloc(sizeof(int) * (size_t)N);
              lead_rec = (int*)malloc(sizeof(int) * (size_t)N);
              lead_dist = (double*)malloc(sizeof(double) * (size_t)N);
            }
            lead_plane[nlead] = m;
            lead_rec[nlead] = (int)((i - r0) * (N - 1) + (j < i ? j : j - 1));
            lead_dist[nlead] = 0.5 * rec.dist;
            nlead++;
          }
        }
        if (have || !(rec.flags & LQRO_REC_STALE)) {
          for (int k = 0; k < 3; k++) cur[k] = rec.normal[k];
          have = 1;
        }
      }
      if (recs) recs[(size_t)(i - r0) * (N - 1) + (j < i ? j : j - 1)] = rec;
      if (rec.flags & LQRO_REC_PLANE) {
        for (int k = 0; k < 3; k++) {
          planes[6 * m + k] = rec.plane_point[k];
          planes[6 * m + 3 + k] = rec.plane_normal[k];
        }
        m++;
      }
    }
    if (rs) {
      rowstate_t* R = &rs[i - r0];
      R->kind = have ? 1 : (nlead ? 2 : 0);
      for (int k = 0; k < 3; k++) R->last[k] = cur[k];
      R->m = m;
      R->nlead = nlead;
      if (nlead) {   /* the LP waits for the previous row's normal (resolve_rows) */
        R->planes = (float*)malloc(sizeof(float) * 6 * (size_t)(m ? m : 1));
        memcpy(R->planes, planes, sizeof(float) * 6 * (size_t)m);
        R->lead_plane = lead_plane; R->lead_rec = lead_rec; R->lead_dist = lead_dist;
        continue;
      }
      free(lead_plane); free(lead_rec); free(lead_dist);
    }
    orc_newv(m, planes, vgoal + (size_t)i * 3, vmax_lp, newv + (size_t)i * 3);  /* LQRO:1435 */
  }
out:
  free(pts); free(planes); free(sel); free(Tf); free(Nf);
  return rc;
}

/* The rows in order (LQRO:1393): leading stale pairs take the normal the
 * previous row left (g_carry for the first row), then the row's LP runs;
 * g_carry leaves with the last row's normal, for the next step. */
static void resolve_rows(int N, int X, double vmax_lp, const double* x, const double* vgoal, int r0, int r1,
                         double* newv, lqro_pair_record* recs, rowstate_t* rs) {
  double carry[3] = {g_carry[0], g_carry[1], g_carry[2]};
  for (int i = r0; i < r1; ++i) {
    rowstate_t* R = &rs[i - r0];
    if (R->nlead) {
      for (int q = 0; q < R->nlead; q++) {
        float* pl = R->planes + 6 * (size_t)R->lead_plane[q];
        stale_plane(x + (size_t)i * X, R->lead_dist[q], carry, pl, pl + 3);
        if (recs) {
          lqro_pair_record* r = &recs[R->lead_rec[q]];
          for (int k = 0; k < 3; k++) {
            r->normal[k] = carry[k];
            r->plane_point[k] = pl[k];
            r->plane_normal[k] = pl[3 + k];
          }
        }
      }
      orc_newv(R->m, R->planes, vgoal + (size_t)i * 3, vmax_lp, newv + (size_t)i * 3);   /* LQRO:1435 */
      free(R->planes); free(R->lead_plane); free(R->lead_rec); free(R->lead_dist);
    }
    if (R->kind == 1)
      for (int k = 0; k < 3; k++) carry[k] = R->last[k];
  }
  for (int k = 0; k < 3; k++) g_carry[k] = carry[k];
}

int orc_step(int N, int X, int H, int NP, int min_reach, double vmax_reach, double vmax_lp,
             int per_agent, const double* T, const double* NCF, const double* S,
             const double* x, const double* vgoal, int r0, int r1, double* newv,
             lqro_pair_record* recs) {
  rowstate_t* rs = g_hull_rule ? (rowstate_t*)calloc((size_t)(r1 - r0 > 0 ? r1 - r0 : 1), sizeof(rowstate_t)) : NULL;
  int rc = step_rows(N, X, H, NP, min_reach, vmax_reach, vmax_lp, per_agent, T, NCF, S, x, vgoal, r0,
                     r1, newv, recs, NULL, rs);
  if (rs && !rc) resolve_rows(N, X, vmax_lp, x, vgoal, r0, r1, newv, recs, rs);
  free(rs);
  return rc;
}

typedef struct {
  int N, X, H, NP, min_reach, per_agent, r0, r1, rc;
  double vmax_reach, vmax_lp;
  const double *T, *NCF, *S, *x, *vgoal;
  double* newv;
  lqro_pair_record* recs;
  int rbase;
  const faith_t* fa;
  rowstate_t* rs;
} mt_arg;

static void* mt_body(void* p) {
  mt_arg* a = (mt_arg*)p;
  a->rc = step_rows(a->N, a->X, a->H, a->NP, a->min_reach, a->vmax_reach, a->vmax_lp, a->per_agent,
                    a->T, a->NCF, a->S, a->x, a->vgoal, a->r0, a->r1, a->newv,
                    a->recs ? a->recs + (size_t)(a->r0 - a->rbase) * (a->N - 1) : NULL, a->fa,
                    a->rs ? a->rs + (a->r0 - a->rbase) : NULL);
  return NULL;
}

static int step_mt(int N, int X, int H, int NP, int min_reach, double vmax_reach, double vmax_lp,
                   int per_agent, const double* T, const double* NCF, const double* S,
                   const double* x, const double* vgoal, int r0, int r1, double* newv,
                   lqro_pair_record* recs, int threads, const faith_t* fa);

int orc_step_mt(int N, int X, int H, int NP, int min_reach, double vmax_reach, double vmax_lp,
                int per_agent, const double* T, const double* NCF, const double* S,
                const double* x, const double* vgoal, int r0, int r1, double* newv,
                lqro_pair_record* recs, int threads) {
  return step_mt(N, X, H, NP, min_reach, vmax_reach, vmax_lp, per_agent, T, NCF, S, x, vgoal, r0, r1,
                 newv, recs, threads, NULL);
}

/* The reference-faithful step: the pair loop with the reference's per-pair
 * cost structure (findFG recursion per pair, LQRO:1401-1406; GJK twice for
 * an outside pair, LQRO:1410/1414); results bit-identical to orc_step_mt.
 * The CPU baseline bench.py times. */
int orc_step_faithful_mt(int N, int X, int H, int NP, int min_reach, double vmax_reach,
                         double vmax_lp, int per_agent, const double* A, const double* B,
                         const double* L, const double* E, const double* S, const double* x,
                         const double* vgoal, int r0, int r1, double* newv,
                         lqro_pair_record* recs, int threads) {
  faith_t fa = {A, B, L, E};
  return step_mt(N, X, H, NP, min_reach, vmax_reach, vmax_lp, per_agent, NULL, NULL, S, x, vgoal, r0,
                 r1, newv, recs, threads, &fa);
}

static int step_mt(int N, int X, int H, int NP, int min_reach, double vmax_reach, double vmax_lp,
                   int per_agent, const double* T, const double* NCF, const double* S,
                   const double* x, const double* vgoal, int r0, int r1, double* newv,
                   lqro_pair_record* recs, int threads, const faith_t* fa) {
  rowstate_t* rs = g_hull_rule ? (rowstate_t*)calloc((size_t)(r1 - r0 > 0 ? r1 - r0 : 1), sizeof(rowstate_t)) : NULL;
  if (threads <= 1) {
    int rc1 = step_rows(N, X, H, NP, min_reach, vmax_reach, vmax_lp, per_agent, T, NCF, S, x, vgoal, r0,
                        r1, newv, recs, fa, rs);
    if (rs && !rc1) resolve_rows(N, X, vmax_lp, x, vgoal, r0, r1, newv, recs, rs);
    free(rs);
    return rc1;
  }
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)threads);
  mt_arg* args = (mt_arg*)malloc(sizeof(mt_arg) * (size_t)threads);
  int rows = r1 - r0, rc = 0;
  for (int t = 0; t < threads; t++) {
    mt_arg* a = &args[t];
    a->N = N; a->X = X; a->H = H; a->NP = NP; a->min_reach = min_reach; a->per_agent = per_agent;
    a->vmax_reach = vmax_reach; a->vmax_lp = vmax_lp; a->T = T; a->NCF = NCF; a->S = S; a->x = x;
    a->vgoal = vgoal; a->newv = newv; a->recs = recs; a->rbase = r0; a->fa = fa; a->rs = rs;
    a->r0 = r0 + (int)((long long)rows * t / threads);
    a->r1 = r0 + (int)((long long)rows * (t + 1) / threads);
    a->rc = 0;
    pthread_create(&th[t], NULL, mt_body, a);
  }
  for (int t = 0; t < threads; t++) { pthread_join(th[t], NULL); if (args[t].rc) rc = args[t].rc; }
  free(th); free(args);
  if (rs && !rc) resolve_rows(N, X, vmax_lp, x, vgoal, r0, r1, newv, recs, rs);
  free(rs);
  return rc;
}

/* ------------------------------------------------------------------------ */
/* The per-agent step after the pair loop (LQRO:1437-1446): findU, propagate, */
/* kalmanFilter1, the observation draw, kalmanFilter2, findVGoal.  Noise      */
/* draws are supplied (16 for propagate, 6 for the observation).              */
/* ------------------------------------------------------------------------ */

/* jacobi (MAT:674-759) */
static void ojacobi(int n, const double* m, double* V, double* D) {
  memcpy(D, m, sizeof(double) * (size_t)(n * n));
  meye(n, V);
  if (n <= 1) return;
  size_t pivotRow = 0, zeroCount = 0;
  for (;;) {
    double maximum = 0;
    size_t p = 0, q = 0;
    for (size_t i = 0; i < pivotRow; ++i)
      if (fabs(D[i * n + pivotRow]) > maximum) {
        maximum = fabs(D[i * n + pivotRow]); p = i; q = pivotRow;
      }
    for (size_t j = pivotRow + 1; j < (size_t)n; ++j)
      if (fabs(D[pivotRow * n + j]) > maximum) {
        maximum = fabs(D[pivotRow * n + j]); p = pivotRow; q = j;
      }
    pivotRow = (pivotRow + 1) % (size_t)n;
    if (maximum <= 2.220446049250313080847e-16) {   /* DBL_EPSILON */
      ++zeroCount;
      if (zeroCount == (size_t)n) break;
      continue;
    }
    zeroCount = 0;
    double theta = 0.5 * (D[q * n + q] - D[p * n + p]) / D[p * n + q];
    double t = 1 / (fabs(theta) + hypot(theta, 1));
    if (theta < 0) t = -t;
    double c = 1 / hypot(t, 1);
    double s = c * t;
    double tau = s / (1 + c);
    for (size_t r = 0; r < p; ++r) {
      double Drp = D[r * n + p], Drq = D[r * n + q];
      D[r * n + p] -= s * (Drq + tau * Drp);
      D[r * n + q] += s * (Drp - tau * Drq);
    }
    for (size_t r = p + 1; r < q; ++r) {
      double Drp = D[p * n + r], Drq = D[r * n + q];
      D[p * n + r] -= s * (Drq + tau * Drp);
      D[r * n + q] += s * (Drp - tau * Drq);
    }
    for (size_t r = q + 1; r < (size_t)n; ++r) {
      double Drp = D[p * n + r], Drq = D[q * n + r];
      D[p * n + r] -= s * (Drq + tau * Drp);
      D[q * n + r] += s * (Drp - tau * Drq);
    }
    D[p * n + p] -= t * D[p * n + q];
    D[q * n + q] += t * D[p * n + q];
    D[p * n + q] = 0;
    for (size_t r = 0; r < (size_t)n; ++r) {
      double Vrp = V[r * n + p], Vrq = V[r * n + q];
      V[r * n + p] -= s * (Vrq + tau * Vrp);
      V[r * n + q] += s * (Vrp - tau * Vrq);
    }
  }
  for (int i = 0; i < n - 1; ++i)
    for (int j = i + 1; j < n; ++j) D[j * n + i] = D[i * n + j] = 0;
}

void orc_jacobi(int n, const double* m, double* V, double* D) { ojacobi(n, m, V, D); }

/* sampleGaussian (simulator2.h:21-32) with the normals supplied */
static void sample_gauss(int n, const double* mean, const double* var, const double* nrm,
                         double* out) {
  double V[MXN * MXN], D[MXN * MXN], VD[MXN * MXN], t[MXN];
  ojacobi(n, var, V, D);
  for (int i = 0; i < n; ++i) D[i * n + i] = sqrt(D[i * n + i]);
  mm(n, n, n, V, D, VD);
  mm(n, n, 1, VD, nrm, t);
  madd(n, t, mean, out);
}

/* h (LQRO:399-419) */
static void obs_h(const double* x, double* z) {
  z[0] = x[9]; z[1] = x[10]; z[2] = x[11];
  z[3] = x[0]; z[4] = x[1]; z[5] = x[2];
}

/* errFromRot (stdafx.h:35-48) */
static void err_from_rot(const double* R, double* out) {
  double q[3] = {R[7] - R[5], R[2] - R[6], R[3] - R[1]};
  double r = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2]);
  double t = R[0] + R[4] + R[8] - 1;
  if (r == 0) { out[0] = out[1] = out[2] = 0.0; return; }
  mscale(3, q, atan2(r, t) / r, out);
}

/* the yaw-only frame RLocal and xTilde of both controllers (LQRO:597-616) */
static void ctrl_frame(const double* x, const double* R0, const double* uGoal, double* RL,
                       double* xt) {
  double z0[3] = {R0[2], R0[5], R0[8]}, ez[3] = {0, 0, 1}, S[9], axis[3];
  skew(z0, S);
  mm(3, 3, 1, S, ez, axis);
  double sinangle = sqrt(axis[0] * axis[0] + axis[1] * axis[1] + axis[2] * axis[2]);
  double angle = asin(sinangle);
  if (sinangle != 0) mscale(3, axis, angle / sinangle, axis);
  double Sa[9], Ea[9], RLt[9], RR[9];
  skew(axis, Sa); mexp(3, Sa, Ea); mm(3, 3, 3, Ea, R0, RL);
  mt(3, 3, RL, RLt);
  mm(3, 3, 1, RLt, x, xt);          /* position */
  mm(3, 3, 1, RLt, x + 3, xt + 3);  /* velocity */
  mm(3, 3, 3, RLt, R0, RR);
  err_from_rot(RR, xt + 6);
  xt[9] = x[9]; xt[10] = x[10]; xt[11] = x[11];
  for (int k = 0; k < 4; ++k) xt[12 + k] = x[12 + k] - uGoal[k];
}

/* riccatiControllerSteady (LQRO:594-617) */
void orc_control_velocity(const double* x, const double* R0, const double* vGoal,
                          const double* uGoal, const double* L, const double* E,
                          const double* l, double* u) {
  double RL[9], RLt[9], xt[16], vt[3], Lx[4], Ev[4];
  ctrl_frame(x, R0, uGoal, RL, xt);
  mt(3, 3, RL, RLt);
  mm(3, 3, 1, RLt, vGoal, vt);
  mm(4, 16, 1, L, xt, Lx);
  mm(4, 3, 1, E, vt, Ev);
  madd(4, uGoal, Lx, u); madd(4, u, Ev, u); madd(4, u, l, u);
}

/* riccatiControllerSteadyPosition (LQRO:619-645) */
void orc_control_position(const double* x, const double* R0, const double* pGoal,
                          const double* uGoal, const double* Lh, const double* Eh, double* v) {
  double RL[9], RLt[9], xt[16], pt[3], a[3], b[3];
  ctrl_frame(x, R0, uGoal, RL, xt);
  mt(3, 3, RL, RLt);
  mm(3, 3, 1, RLt, pGoal, pt);
  mm(3, 16, 1, Lh, xt, a);
  mm(3, 3, 1, Eh, pt, b);
  madd(3, a, b, a);
  mm(3, 3, 1, RL, a, v);
}

/* the common head of propagate and kalmanFilter1 (LQRO:474-481, 489-500) */
static void disc_step(const phys_t* P, const double* x, const double* R, const double* u,
                      const double* M, double* A, double* MM, double* dx) {
  enum { X = 16 };
  double F[X * X], xdot[X], fr[X], fl[X], xr[X], xl[X];
  memcpy(xr, x, sizeof xr); memcpy(xl, x, sizeof xl);
  for (int i = 0; i < X; ++i) {       /* Jacobian_fx (LQRO:421-430) */
    xr[i] += P->jStep; xl[i] -= P->jStep;
    fdyn(P, xr, R, u, fr); fdyn(P, xl, R, u, fl);
    for (int k = 0; k < X; ++k) F[k * X + i] = (fr[k] - fl[k]) / (2 * P->jStep);
    xr[i] = xl[i] = x[i];
  }
  fdyn(P, x, R, u, xdot);
  double t[X * X], A2[X * X], t2[X * X], t3[X * X], At[X * X], A2t[X * X];
  mscale(X * X, F, P->dt, t); mexp(X, t, A);
  mscale(X * X, F, P->dt * 0.5, t); mexp(X, t, A2);
  /* MM = (dt/6) * (M + 4*A2*M*~A2 + A*M*~A) */
  mt(X, X, A2, A2t); mt(X, X, A, At);
  mscale(X * X, A2, 4, t); mm(X, X, X, t, M, t2); mm(X, X, X, t2, A2t, t2);
  madd(X * X, M, t2, t3);
  mm(X, X, X, A, M, t2); mm(X, X, X, t2, At, t2);
  madd(X * X, t3, t2, t3);
  mscale(X * X, t3, P->dt / 6, MM);
  /* dx = (dt/6)*(xDot + 4*(A2*xDot) + A*xDot) */
  double a[X], b[X];
  mm(X, X, 1, A2, xdot, a); mscale(X, a, 4, a);
  madd(X, xdot, a, a);
  mm(X, X, 1, A, xdot, b); madd(X, a, b, a);
  mscale(X, a, P->dt / 6, dx);
}

static void rot_reset(double* x, double* R) {     /* LQRO:483-485 */
  double S[9], E[9];
  skew(x + 6, S); mexp(3, S, E); mm(3, 3, 3, R, E, R);
  x[6] = 0; x[7] = 0; x[8] = 0;
}

/* propagate (LQRO:473-486) */
void orc_propagate(const lqro_model* m, double* x, double* R, const double* u, const double* M,
                   const double* nrm) {
  phys_t P; phys_init(m, &P);
  double A[256], MM[256], dx[16], zero[16] = {0}, g[16];
  disc_step(&P, x, R, u, M, A, MM, dx);
  sample_gauss(16, zero, MM, nrm, g);
  madd(16, x, dx, x); madd(16, x, g, x);
  rot_reset(x, R);
}

/* kalmanFilter1 (LQRO:488-505) */
void orc_kalman1(const lqro_model* m, double* x, double* R, const double* u, const double* M,
                 double* Pc) {
  phys_t P; phys_init(m, &P);
  double A[256], MM[256], dx[16], At[256], t[256];
  disc_step(&P, x, R, u, M, A, MM, dx);
  madd(16, x, dx, x);
  mt(16, 16, A, At);
  mm(16, 16, 16, A, Pc, t); mm(16, 16, 16, t, At, t); madd(256, t, MM, Pc);
  rot_reset(x, R);
}

/* kalmanFilter2 (LQRO:507-518) with Jacobian_hx (LQRO:443-452) */
void orc_kalman2(const lqro_model* m, double* x, double* R, const double* z, const double* Nz,
                 double* Pc) {
  enum { X = 16, Z = 6 };
  phys_t P; phys_init(m, &P);
  double H[Z * X], xr[X], xl[X], hr[Z], hl[Z];
  memcpy(xr, x, sizeof xr); memcpy(xl, x, sizeof xl);
  for (int i = 0; i < X; ++i) {
    xr[i] += P.jStep; xl[i] -= P.jStep;
    obs_h(xr, hr); obs_h(xl, hl);
    for (int k = 0; k < Z; ++k) H[k * X + i] = (hr[k] - hl[k]) / (2 * P.jStep);
    xr[i] = xl[i] = x[i];
  }
  double Ht[X * Z], PHt[X * Z], HP[Z * X], S[Z * Z], Si[Z * Z], K[X * Z];
  mt(Z, X, H, Ht);
  mm(X, X, Z, Pc, Ht, PHt);
  mm(Z, X, X, H, Pc, HP); mm(Z, X, Z, HP, Ht, S); madd(Z * Z, S, Nz, S);
  minv(Z, S, Si);
  mm(X, Z, Z, PHt, Si, K);
  double hx[Z], e[Z], Ke[X];
  obs_h(x, hx); msub(Z, z, hx, e);
  mm(X, Z, 1, K, e, Ke); madd(X, x, Ke, x);
  double KH[X * X], I[X * X];
  mm(X, Z, X, K, H, KH); meye(X, I); msub(X * X, I, KH, I);
  mm(X, X, X, I, Pc, Pc);
  rot_reset(x, R);
}

/* One agent through LQRO:1438-1445 (see lqro_oracle.h). */
void orc_agent_step(const lqro_model* m, const double* L, const double* E, const double* l,
                    const double* Lh, const double* Eh, const double* uGoal, const double* pGoal,
                    const double* M, const double* Nz, const double* nrm, double* x, double* R,
                    double* xTrue, double* RTrue, double* Pc, double* vgoal, double* u_out) {
  double u[4], z[6], hz[6];
  orc_control_velocity(x, R, vgoal, uGoal, L, E, l, u);     /* findU (vGoal = newV) */
  orc_propagate(m, xTrue, RTrue, u, M, nrm);                /* propagateU */
  orc_kalman1(m, x, R, u, M, Pc);
  obs_h(xTrue, hz);
  sample_gauss(6, hz, Nz, nrm + 16, z);                     /* LQRO:1442 */
  orc_kalman2(m, x, R, z, Nz, Pc);
  orc_control_position(x, R, pGoal, uGoal, Lh, Eh, vgoal);  /* findVGoal */
  if (u_out) memcpy(u_out, u, sizeof u);
}

/* quatFromRot (stdafx.h:24-33) and Quadrotor::visualize's keyframe
 * (LQRO:128-133): (float) t, (float) xTrue[0..2], (float) quat */
void orc_quat_from_rot(const double* R, double* q) {
  double a;
  a = 1 + R[0] - R[4] - R[8]; q[0] = 0.5 * sqrt(a < 0.0 ? 0.0 : a) * (R[7] - R[5] >= 0 ? 1 : -1);
  a = 1 - R[0] + R[4] - R[8]; q[1] = 0.5 * sqrt(a < 0.0 ? 0.0 : a) * (R[2] - R[6] >= 0 ? 1 : -1);
  a = 1 - R[0] - R[4] + R[8]; q[2] = 0.5 * sqrt(a < 0.0 ? 0.0 : a) * (R[3] - R[1] >= 0 ? 1 : -1);
  a = 1 + R[0] + R[4] + R[8]; q[3] = 0.5 * sqrt(a < 0.0 ? 0.0 : a);
}

void orc_keyframe(double t, const double* xTrue, const double* RTrue, float* out) {
  double q[4];
  orc_quat_from_rot(RTrue, q);
  out[0] = (float)t;
  for (int k = 0; k < 3; ++k) out[1 + k] = (float)xTrue[k];
  for (int k = 0; k < 4; ++k) out[4 + k] = (float)q[k];
}
