/* fcl_gjk_indep.h -- TEST INFRASTRUCTURE (the CPU oracle's checker; never
 * linked into the product).  Included by collide_oracle.c.
 *
 * fcl::collide with CollisionRequest(gjk_solver_type = GST_INDEP) on a shape
 * pair that has no closed form: GJKSolver_indep::shapeIntersect ->
 * ShapeIntersectIndepImpl (generic) -> details::GJK::evaluate on a
 * details::MinkowskiDiff [ext FCL 0.7.0: fcl/narrowphase/detail/gjk_solver_indep-inl.h,
 * convexity_based_algorithm/gjk-inl.h, minkowski_diff-inl.h,
 * fcl/math/detail/project-inl.h].  FCL is not under /root/reference:
 * restated from FCL 0.7.0's published source, parity with FCL unpinned beyond
 * the geometric known answers (tests/test_gjk_indep.py).
 *
 *   guess = (1, 0, 0) (enable_cached_guess false); shapes[0] = s1,
 *   shapes[1] = s2; toshape1 = R2^T R1; toshape0 = tf1^-1 tf2 (Isometry:
 *   R1^T R2, R1^T t2 + (-(R1^T t1))); GJK(max_iterations 128, tolerance =
 *   the request's gjk_tolerance) evaluate(shape, -guess): collision iff the
 *   status is Inside.  Everything in double, in s1's frame:
 *   support(d) = support0(d) - support1(-d), support0(d) = getSupport(s1, d),
 *   support1(d) = toshape0 * getSupport(s2, toshape1 * d); GJK::getSupport
 *   normalises d first.
 * getSupport (gjk-inl.h): box (d_i > 0 ? side_i / 2 : -side_i / 2); sphere
 * d * r; capsule pos1/pos2 = (0, 0, +-lz/2) + d * r, the larger d . pos;
 * cylinder zdist = sqrt(d0^2 + d1^2), zdist == 0 -> (0, 0, +-lz/2) else
 * (r/zdist d0, r/zdist d1, +-lz/2); cone: the apex (0, 0, lz/2) when
 * d2 > |d| sin a (sin a = r / sqrt(r^2 + 4 (lz/2)^2)), else the rim point
 * (r/zdist d0, r/zdist d1, -lz/2), else (0, 0, -lz/2); ellipsoid v / sqrt(v . d)
 * with v = (a^2 d0, b^2 d1, c^2 d2); triangle (TriangleP) the first of the
 * larger d . a / d . b / d . c; convex Convex::findExtremeVertex (the
 * neighbour walk on watertight hulls of more than 32 vertices, else the
 * first maximum) -- convex_find_extreme above.
 * Eigen's 3-term sums are taken in the oracle's default order
 * ((x0 + x1) + x2), as everywhere in this file. */
#ifndef FCL_GJK_INDEP_H
#define FCL_GJK_INDEP_H

typedef struct { real v[3]; } gv3;

static inline gv3 gv(real x, real y, real z) { gv3 r = {{x, y, z}}; return r; }
static inline gv3 gadd(gv3 a, gv3 b) { return gv(a.v[0] + b.v[0], a.v[1] + b.v[1], a.v[2] + b.v[2]); }
static inline gv3 gsub(gv3 a, gv3 b) { return gv(a.v[0] - b.v[0], a.v[1] - b.v[1], a.v[2] - b.v[2]); }
static inline gv3 gscale(gv3 a, real s) { return gv(a.v[0] * s, a.v[1] * s, a.v[2] * s); }
static inline real gdot(gv3 a, gv3 b) { return (a.v[0] * b.v[0] + a.v[1] * b.v[1]) + a.v[2] * b.v[2]; }
static inline real gnorm2(gv3 a) { return gdot(a, a); }
static inline gv3 gcross(gv3 a, gv3 b) {
    return gv(a.v[1] * b.v[2] - a.v[2] * b.v[1], a.v[2] * b.v[0] - a.v[0] * b.v[2], a.v[0] * b.v[1] - a.v[1] * b.v[0]);
}
static inline real gtriple(gv3 a, gv3 b, gv3 c) { return gdot(a, gcross(b, c)); }
/* 3x3 (row-major) times vector */
static inline gv3 gmatv(const real *M, gv3 d) {
    return gv((M[0] * d.v[0] + M[1] * d.v[1]) + M[2] * d.v[2], (M[3] * d.v[0] + M[4] * d.v[1]) + M[5] * d.v[2],
              (M[6] * d.v[0] + M[7] * d.v[1]) + M[8] * d.v[2]);
}

/* ---------------------------------------------------------- Project<S> */
typedef struct {
    real param[4];
    unsigned encode;
    real sqr_distance;
} gproj;

static gproj gproj_init(void) {
    gproj r;
    r.param[0] = r.param[1] = r.param[2] = r.param[3] = 0.0;
    r.encode = 0;
    r.sqr_distance = -1.0;
    return r;
}

/* Project<S>::projectLineOrigin */
static gproj project_line_origin(gv3 a, gv3 b) {
    gproj res = gproj_init();
    const gv3 d = gsub(b, a);
    const real l = gnorm2(d);
    if (l > 0) {
        const real t = -gdot(a, d);
        res.param[1] = (t >= l) ? 1.0 : ((t <= 0) ? 0.0 : (t / l));
        res.param[0] = 1 - res.param[1];
        if (t >= l) {
            res.sqr_distance = gnorm2(b);
            res.encode = 2;
        } else if (t <= 0) {
            res.sqr_distance = gnorm2(a);
            res.encode = 1;
        } else {
            res.sqr_distance = gnorm2(gadd(a, gscale(d, res.param[1])));
            res.encode = 3;
        }
    }
    return res;
}

/* Project<S>::projectTriangleOrigin */
static gproj project_triangle_origin(gv3 a, gv3 b, gv3 c) {
    gproj res = gproj_init();
    static const int nexti[3] = {1, 2, 0};
    const gv3 vt[3] = {a, b, c};
    const gv3 dl[3] = {gsub(a, b), gsub(b, c), gsub(c, a)};
    const gv3 n = gcross(dl[0], dl[1]);
    const real l = gnorm2(n);
    if (l > 0) {
        real mindist = -1;
        for (int i = 0; i < 3; ++i) {
            if (gdot(vt[i], gcross(dl[i], n)) > 0) {
                const int j = nexti[i];
                const gproj rl = project_line_origin(vt[i], vt[j]);
                if (mindist < 0 || rl.sqr_distance < mindist) {
                    mindist = rl.sqr_distance;
                    res.encode = ((rl.encode & 1) ? 1u << i : 0u) + ((rl.encode & 2) ? 1u << j : 0u);
                    res.param[i] = rl.param[0];
                    res.param[j] = rl.param[1];
                    res.param[nexti[j]] = 0;
                }
            }
        }
        if (mindist < 0) {
            const real d = gdot(a, n);
            const real s = sqrt(l);
            const gv3 p = gscale(n, d / l);
            mindist = gnorm2(p);
            res.encode = 7;
            res.param[0] = sqrt(gnorm2(gcross(dl[1], gsub(b, p)))) / s;
            res.param[1] = sqrt(gnorm2(gcross(dl[2], gsub(c, p)))) / s;
            res.param[2] = 1 - res.param[0] - res.param[1];
        }
        res.sqr_distance = mindist;
    }
    return res;
}

/* Project<S>::projectTetrahedraOrigin */
static gproj project_tetrahedra_origin(gv3 a, gv3 b, gv3 c, gv3 d) {
    gproj res = gproj_init();
    static const int nexti[3] = {1, 2, 0};
    const gv3 vt[4] = {a, b, c, d};
    const gv3 dl[3] = {gsub(a, d), gsub(b, d), gsub(c, d)};
    const real vl = gtriple(dl[0], dl[1], dl[2]);
    const int ng = (vl * gdot(a, gcross(gsub(b, c), gsub(a, b)))) <= 0;
    if (ng && fabs(vl) > 0) {
        real mindist = -1;
        for (int i = 0; i < 3; ++i) {
            const int j = nexti[i];
            const real s = vl * gdot(d, gcross(dl[i], dl[j]));
            if (s > 0) {
                const gproj rt = project_triangle_origin(vt[i], vt[j], d);
                if (mindist < 0 || rt.sqr_distance < mindist) {
                    mindist = rt.sqr_distance;
                    res.encode = ((rt.encode & 1) ? 1u << i : 0u) + ((rt.encode & 2) ? 1u << j : 0u) +
                                 ((rt.encode & 4) ? 8u : 0u);
                    res.param[i] = rt.param[0];
                    res.param[j] = rt.param[1];
                    res.param[nexti[j]] = 0;
                    res.param[3] = rt.param[2];
                }
            }
        }
        if (mindist < 0) {
            mindist = 0;
            res.encode = 15;
            res.param[0] = gtriple(c, b, d) / vl;
            res.param[1] = gtriple(a, c, d) / vl;
            res.param[2] = gtriple(b, a, d) / vl;
            res.param[3] = 1 - (res.param[0] + res.param[1] + res.param[2]);
        }
        res.sqr_distance = mindist;
    } else if (!ng) {
        res = project_triangle_origin(a, b, c);
        res.param[3] = 0;
    }
    return res;
}

/* ------------------------------------------------------ MinkowskiDiff */
typedef struct {
    int type;
    const real *prm;    /* geom_param: box sides / radius / (radius, lz) */
    const real *verts;  /* convex */
    int nv;
    const int *nbr;
} gshape;

typedef struct {
    gshape s[2];
    real toshape1[9];    /* R2^T R1 */
    real toshape0_R[9];  /* R1^T R2 */
    real toshape0_t[3];  /* R1^T t2 + (-(R1^T t1)) */
} gmink;

/* getSupport (gjk-inl.h) in the shape's own frame */
static gv3 gjk_shape_support(const gshape *sh, gv3 d) {
    switch (sh->type) {
    case GEOM_BOX:
        return gv((d.v[0] > 0) ? (sh->prm[0] / 2) : (-sh->prm[0] / 2), (d.v[1] > 0) ? (sh->prm[1] / 2) : (-sh->prm[1] / 2),
                  (d.v[2] > 0) ? (sh->prm[2] / 2) : (-sh->prm[2] / 2));
    case GEOM_SPHERE:
        return gscale(d, sh->prm[0]);
    case GEOM_CAPSULE: {
        const real half_h = sh->prm[1] * 0.5;
        gv3 pos1 = gv(0, 0, half_h), pos2 = gv(0, 0, -half_h);
        const gv3 v = gscale(d, sh->prm[0]);
        pos1 = gadd(pos1, v);
        pos2 = gadd(pos2, v);
        return gdot(d, pos1) > gdot(d, pos2) ? pos1 : pos2;
    }
    case GEOM_CYLINDER: {
        const real zdist = sqrt(d.v[0] * d.v[0] + d.v[1] * d.v[1]);
        const real half_h = sh->prm[1] * 0.5;
        if (zdist == 0.0) return gv(0, 0, (d.v[2] > 0) ? half_h : -half_h);
        const real dd = sh->prm[0] / zdist;
        return gv(dd * d.v[0], dd * d.v[1], (d.v[2] > 0) ? half_h : -half_h);
    }
    case GEOM_CONE: {
        real zdist = d.v[0] * d.v[0] + d.v[1] * d.v[1];
        real len = zdist + d.v[2] * d.v[2];
        zdist = sqrt(zdist);
        len = sqrt(len);
        const real half_h = sh->prm[1] * 0.5, radius = sh->prm[0];
        const real sin_a = radius / sqrt(radius * radius + 4 * half_h * half_h);
        if (d.v[2] > len * sin_a) return gv(0, 0, half_h);
        if (zdist > 0) {
            const real rad = radius / zdist;
            return gv(rad * d.v[0], rad * d.v[1], -half_h);
        }
        return gv(0, 0, -half_h);
    }
    case GEOM_TRIANGLE_P: { /* the first of the larger dot products a / b / c */
        const gv3 a = gv(sh->verts[0], sh->verts[1], sh->verts[2]), b = gv(sh->verts[3], sh->verts[4], sh->verts[5]),
                  c = gv(sh->verts[6], sh->verts[7], sh->verts[8]);
        const real dota = gdot(d, a), dotb = gdot(d, b), dotc = gdot(d, c);
        if (dota > dotb) return dotc > dota ? c : a;
        return dotc > dotb ? c : b;
    }
    case GEOM_ELLIPSOID: { /* v / sqrt(v . d): Eigen's quotient, one division per coefficient */
        const real a2 = sh->prm[0] * sh->prm[0], b2 = sh->prm[1] * sh->prm[1], c2 = sh->prm[2] * sh->prm[2];
        const gv3 v = gv(a2 * d.v[0], b2 * d.v[1], c2 * d.v[2]);
        const real dd = sqrt(gdot(v, d));
        return gv(v.v[0] / dd, v.v[1] / dd, v.v[2] / dd);
    }
    default: { /* GEOM_CONVEX */
        const real dC[3] = {d.v[0], d.v[1], d.v[2]};
        const int k = convex_find_extreme(sh->verts, sh->nv, sh->nbr, dC, NULL);
        return gv(sh->verts[3 * k], sh->verts[3 * k + 1], sh->verts[3 * k + 2]);
    }
    }
}

static gv3 gmink_support(const gmink *m, gv3 d) {
    const gv3 s0 = gjk_shape_support(&m->s[0], d);
    const gv3 l1 = gjk_shape_support(&m->s[1], gmatv(m->toshape1, gscale(d, -1.0)));
    const gv3 s1 = gadd(gmatv(m->toshape0_R, l1), gv(m->toshape0_t[0], m->toshape0_t[1], m->toshape0_t[2]));
    return gsub(s0, s1);
}

/* --------------------------------------------------------------- GJK */
typedef struct { gv3 d, w; } gsv;
typedef struct { gsv *c[4]; real p[4]; int rank; } gsimplex;
enum { GJK_VALID = 0, GJK_INSIDE = 1, GJK_FAILED = 2 };

typedef struct {
    const gmink *shape;
    gsv store[4];
    gsv *free_v[4];
    int nfree;
    gsimplex simplices[2];
} gjk_state;

/* GJK::getSupport: sv.d = d.normalized(); sv.w = shape.support(sv.d) */
static void gjk_get_support(const gjk_state *g, gv3 d, gsv *sv) {
    const real n2 = gnorm2(d);
    sv->d = d;
    /* Eigen normalized(): n / sqrt(z) -- a division of each coefficient */
    if (n2 > 0) {
        const real s = sqrt(n2);
        sv->d = gv(d.v[0] / s, d.v[1] / s, d.v[2] / s);
    }
    sv->w = gmink_support(g->shape, sv->d);
}

static void gjk_append(gjk_state *g, gsimplex *s, gv3 v) {
    s->p[s->rank] = 0;
    s->c[s->rank] = g->free_v[--g->nfree];
    gjk_get_support(g, v, s->c[s->rank++]);
}

static void gjk_remove(gjk_state *g, gsimplex *s) { g->free_v[g->nfree++] = s->c[--s->rank]; }

/* the simplex GJK<S>::evaluate leaves (getSimplex()): directions and weights */
typedef struct { int rank; gv3 d[4]; real p[4]; } gsimplex_out;

/* GJK<S>::evaluate -> status; *out (may be NULL) = simplices[current] at exit */
static int gjk_evaluate(const gmink *shape, gv3 guess, real tolerance, unsigned max_iterations, gsimplex_out *out) {
    gjk_state g;
    unsigned iterations = 0;
    real alpha = 0;
    gv3 lastw[4];
    unsigned clastw = 0;
    g.shape = shape;
    for (int i = 0; i < 4; ++i) g.free_v[i] = &g.store[i];
    g.nfree = 4;
    int current = 0, status = GJK_VALID;
    g.simplices[0].rank = 0;
    gv3 ray = guess;
    gjk_append(&g, &g.simplices[0], gnorm2(ray) > 0 ? gscale(ray, -1.0) : gv(1, 0, 0));
    g.simplices[0].p[0] = 1;
    ray = g.simplices[0].c[0]->w;
    lastw[0] = lastw[1] = lastw[2] = lastw[3] = ray;
    do {
        const int next = 1 - current;
        gsimplex *curr = &g.simplices[current];
        gsimplex *nxt = &g.simplices[next];
        const real rl = sqrt(gnorm2(ray));
        if (rl < tolerance) {
            status = GJK_INSIDE;
            break;
        }
        gjk_append(&g, curr, gscale(ray, -1.0));
        const gv3 w = curr->c[curr->rank - 1]->w;
        int found = 0;
        for (int i = 0; i < 4; ++i)
            if (gnorm2(gsub(w, lastw[i])) < tolerance) {
                found = 1;
                break;
            }
        if (found) {
            gjk_remove(&g, curr);
            break;
        }
        lastw[clastw = (clastw + 1) & 3] = w;
        const real omega = gdot(ray, w) / rl;
        alpha = alpha > omega ? alpha : omega;
        if ((rl - alpha) - tolerance * rl <= 0) {
            gjk_remove(&g, curr);
            break;
        }
        gproj pr = gproj_init();
        switch (curr->rank) {
        case 2: pr = project_line_origin(curr->c[0]->w, curr->c[1]->w); break;
        case 3: pr = project_triangle_origin(curr->c[0]->w, curr->c[1]->w, curr->c[2]->w); break;
        case 4: pr = project_tetrahedra_origin(curr->c[0]->w, curr->c[1]->w, curr->c[2]->w, curr->c[3]->w); break;
        }
        if (pr.sqr_distance >= 0) {
            nxt->rank = 0;
            ray = gv(0, 0, 0);
            current = next;
            for (int i = 0; i < curr->rank; ++i) {
                if (pr.encode & (1u << i)) {
                    nxt->c[nxt->rank] = curr->c[i];
                    nxt->p[nxt->rank++] = pr.param[i];
                    ray = gadd(ray, gscale(curr->c[i]->w, pr.param[i]));
                } else {
                    g.free_v[g.nfree++] = curr->c[i];
                }
            }
            if (pr.encode == 15) status = GJK_INSIDE;
        } else {
            gjk_remove(&g, curr);
            break;
        }
        status = ((++iterations) < max_iterations) ? status : GJK_FAILED;
    } while (status == GJK_VALID);
    if (out) {
        const gsimplex *fin = &g.simplices[current];
        out->rank = fin->rank;
        for (int i = 0; i < fin->rank; ++i) {
            out->d[i] = fin->c[i]->d;
            out->p[i] = fin->p[i];
        }
    }
    return status;
}

static void gshape_of(const orc_world *w, int geom, gshape *sh) {
    sh->type = w->geom_type[geom];
    sh->prm = w->geom_param + 4 * geom;
    sh->verts = NULL;
    sh->nv = 0;
    sh->nbr = NULL;
    if (sh->type == GEOM_TRIANGLE_P) sh->verts = w->verts + 3 * (size_t)w->geom_vstart[geom];
    if (sh->type == GEOM_CONVEX) {
        sh->verts = w->verts + 3 * (size_t)w->geom_vstart[geom];
        sh->nv = w->geom_nv[geom];
        sh->nbr = (w->conv_nbr && sh->prm[0] >= 0.0) ? w->conv_nbr + (size_t)sh->prm[0] : NULL;
    }
}

static void gmink_of(const orc_world *w, int ga, const real *T1, int gb, const real *T2, gmink *mp) {
    gmink m;
    gshape_of(w, ga, &m.s[0]);
    gshape_of(w, gb, &m.s[1]);
    /* toshape1 = tf2.linear().transpose() * tf1.linear() */
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            m.toshape1[3 * i + j] = (T2[i] * T1[j] + T2[3 + i] * T1[3 + j]) + T2[6 + i] * T1[6 + j];
    /* toshape0 = tf1.inverse(Isometry) * tf2 */
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            m.toshape0_R[3 * i + j] = (T1[i] * T2[j] + T1[3 + i] * T2[3 + j]) + T1[6 + i] * T2[6 + j];
    for (int i = 0; i < 3; ++i) {
        const real inv_t = -((T1[i] * T1[9] + T1[3 + i] * T1[10]) + T1[6 + i] * T1[11]);
        m.toshape0_t[i] = ((T1[i] * T2[9] + T1[3 + i] * T2[10]) + T1[6 + i] * T2[11]) + inv_t;
    }
    *mp = m;
}

/* GJKSolver_indep::shapeIntersect (generic): 1 = collision */
static int gjk_indep_intersect(const orc_world *w, int ga, const real *T1, int gb, const real *T2, real tolerance) {
    gmink m;
    gmink_of(w, ga, T1, gb, T2, &m);
    return gjk_evaluate(&m, gv(-1.0, 0.0, 0.0), tolerance, 128u, NULL) == GJK_INSIDE;
}

/* GJKSolver_indep::shapeDistance (generic, ShapeDistanceIndepImpl): GJK with
 * gjk_tolerance = the request's distance_tolerance; Valid -> w0 = sum p_i
 * support0(d_i), w1 = sum p_i support1(-d_i) (shape 1's frame), distance
 * |w0 - w1|, points tf1 * w0, tf1 * w1; otherwise distance -1 and the points
 * left as the traversal initialised them (zero).  Returns 0. */
static int gjk_indep_distance(const orc_world *w, int ga, const real *T1, int gb, const real *T2, real tolerance,
                              double *dist, double p1[3], double p2[3]) {
    gmink m;
    gsimplex_out s;
    gmink_of(w, ga, T1, gb, T2, &m);
    memset(p1, 0, 3 * sizeof(double));
    memset(p2, 0, 3 * sizeof(double));
    if (gjk_evaluate(&m, gv(-1.0, 0.0, 0.0), tolerance, 128u, &s) != GJK_VALID) {
        *dist = -1.0;
        return 0;
    }
    gv3 w0 = gv(0, 0, 0), w1 = gv(0, 0, 0);
    for (int i = 0; i < s.rank; ++i) {
        const gv3 a = gjk_shape_support(&m.s[0], s.d[i]);
        const gv3 l1 = gjk_shape_support(&m.s[1], gmatv(m.toshape1, gscale(s.d[i], -1.0)));
        const gv3 b = gadd(gmatv(m.toshape0_R, l1), gv(m.toshape0_t[0], m.toshape0_t[1], m.toshape0_t[2]));
        w0 = gadd(w0, gscale(a, s.p[i]));
        w1 = gadd(w1, gscale(b, s.p[i]));
    }
    *dist = sqrt(gnorm2(gsub(w0, w1)));
    for (int i = 0; i < 3; ++i) {
        p1[i] = ((T1[3 * i] * w0.v[0] + T1[3 * i + 1] * w0.v[1]) + T1[3 * i + 2] * w0.v[2]) + T1[9 + i];
        p2[i] = ((T1[3 * i] * w1.v[0] + T1[3 * i + 1] * w1.v[1]) + T1[3 * i + 2] * w1.v[2]) + T1[9 + i];
    }
    return 0;
}

#endif
