/* oracle/fcl_gjk_dist.h -- TEST INFRASTRUCTURE ONLY (included by
 * collide_oracle.c; never linked into the product).
 *
 * FCL 0.7.0's GJK shape distance on libccd, restated operation for operation
 * in ccd_real_t (= float: the reference's libccd 2.1 build):
 *   GJKSolver_libccd::shapeDistance        -> GJKDistance       -> ccdGJKDist2
 *   GJKSolver_libccd::shapeSignedDistance  -> GJKSignedDistance -> ccdGJKSignedDist
 * from FCL's published fcl/narrowphase/detail/convexity_based_algorithm/
 * gjk_libccd-inl.h (namespace libccd_extension: __ccdGJK, doSimplex2/3/4,
 * simplexReduceToTriangle, _ccdDist, extractClosestPoints, __ccdEPA,
 * simplexToPolytope3/4, validateNearestFeatureOfPolytopeBeingEdge,
 * faceNormalPointingOutward, isOutsidePolytopeFace, computeVisiblePatch,
 * expandPolytope, supportEPADirection, nextSupport, penEPAPosClosest) and
 * libccd 2.1's vec3.c (ccdVec3PointSegmentDist2 / ccdVec3PointTriDist2, with
 * and without a witness) and polytope.[ch] (element lists in insertion order,
 * the incremental nearest element, _ccdPtNearestRenew).  Neither FCL nor
 * libccd is under /root/reference: the restatement is written
 * from their published sources and parity with them is UNPINNED beyond the
 * plain-geometry known answers of tests/test_signed_distance.py.
 *
 * Choices where the published code leaves the order to the platform or where
 * this restatement could not be checked against the text:
 *   - expandPolytope iterates std::unordered_set<ccd_pt_edge_t*> (an order
 *     that follows heap addresses); here the border edges are visited in the
 *     order computeVisiblePatch discovers them.  It decides only the list
 *     order of the new edges / faces, i.e. which of several ccdEq-equal
 *     elements _ccdPtNearestUpdate keeps.
 *   - doSimplex2: FCL's rewrite keeps the segment (no "origin beyond A" case,
 *     excluded by GJK's construction) and reports the origin on the segment
 *     when |AB x AO|^2 <= eps^2 |AB|^2 |AO|^2 (eps = float epsilon); the new
 *     direction is libccd's (AB x AO) x AB.
 *   - an enclosing 2-simplex (origin on a segment of the difference) is grown
 *     to a tetrahedron as FCL's convert2SimplexToTetrahedron intends: a
 *     support off the segment, then the farther support along the triangle's
 *     normal; touching (the difference is flat there) reports the segment.
 *   - __ccdEPA: where the nearest face (after
 *     validateNearestFeatureOfPolytopeBeingEdge) is not visible from the new
 *     support point, expandPolytope would delete it all the same (the
 *     visible patch starts there unchecked), the polytope turns non-convex
 *     and the loop can cycle through the same supports without end; the
 *     restatement stops there with that face as the nearest feature (a
 *     "convexity guard", orc_epa_stats counts it: ~1 % of the EPA runs on
 *     the cfg3 / cfg4 test batches).
 *   - _ccdDist: the search direction is taken from a copy of the witness,
 *     so that an iteration whose tetrahedron gives no closer triangle
 *     (simplexReduceToTriangle leaves the witness unset: the new support
 *     was already a simplex vertex) exits with the previous witness, which
 *     lies on the triangle the reduction keeps; the published loop scales
 *     and normalises `dir` in place, which would hand extractClosestPoints
 *     the unit search direction there.  The second exit ("no progress": the
 *     new support point is as far from the origin as the simplex) reports
 *     that support pair (last.v1, last.v2), as libccd's ccdGJKDist2 does.
 * The device twin is mplib_amd/csrc/mpg_kernels.hip (ccd_gjk / ccd_epa); both
 * are compiled without FP contraction and must agree bit for bit.
 */

#define CCD_PT_VERTEX 1
#define CCD_PT_EDGE 2
#define CCD_PT_FACE 3
#define CCD_ZERO CCD_REAL(0.)
#define LX_EPA_TOL CCD_REAL(0.0001) /* CCD_INIT: epa_tolerance */
#define LX_MAX_ITER 1000UL          /* GJKSolver_libccd::max_distance_iterations */
#define LX_THROW (-3)               /* FCL_THROW_FAILED_AT_THIS_CONFIGURATION */

static ccd_real_t lx_dist2(const ccd_vec3_t *a, const ccd_vec3_t *b) {
    ccd_vec3_t ab;
    ccdVec3Sub2(&ab, a, b);
    return ccdVec3Len2(&ab);
}

/* vec3.c __ccdVec3PointSegmentDist2 */
static ccd_real_t lx_seg_dist2(const ccd_vec3_t *P, const ccd_vec3_t *x0, const ccd_vec3_t *b, ccd_vec3_t *witness) {
    ccd_real_t dist, t;
    ccd_vec3_t d, a;
    ccdVec3Sub2(&d, b, x0);
    ccdVec3Sub2(&a, x0, P);
    t = -CCD_REAL(1.) * ccdVec3Dot(&a, &d);
    t /= ccdVec3Len2(&d);
    if (t < CCD_ZERO || ccdIsZero(t)) {
        dist = lx_dist2(x0, P);
        if (witness) ccdVec3Copy(witness, x0);
    } else if (t > CCD_ONE || ccdEq(t, CCD_ONE)) {
        dist = lx_dist2(b, P);
        if (witness) ccdVec3Copy(witness, b);
    } else {
        if (witness) {
            ccdVec3Copy(witness, &d);
            ccdVec3Scale(witness, t);
            ccdVec3Add(witness, x0);
            dist = lx_dist2(witness, P);
        } else {
            ccdVec3Scale(&d, t);
            ccdVec3Add(&d, &a);
            dist = ccdVec3Len2(&d);
        }
    }
    return dist;
}

/* vec3.c ccdVec3PointTriDist2 */
static ccd_real_t lx_tri_dist2(const ccd_vec3_t *P, const ccd_vec3_t *x0, const ccd_vec3_t *B, const ccd_vec3_t *C,
                               ccd_vec3_t *witness) {
    ccd_vec3_t d1, d2, a, witness2;
    ccd_real_t u, v, w, p, q, r, d, s, t, dist, dist2;
    ccdVec3Sub2(&d1, B, x0);
    ccdVec3Sub2(&d2, C, x0);
    ccdVec3Sub2(&a, x0, P);
    u = ccdVec3Dot(&a, &a);
    v = ccdVec3Dot(&d1, &d1);
    w = ccdVec3Dot(&d2, &d2);
    p = ccdVec3Dot(&a, &d1);
    q = ccdVec3Dot(&a, &d2);
    r = ccdVec3Dot(&d1, &d2);
    d = w * v - r * r;
    if (ccdIsZero(d)) {
        s = t = -CCD_REAL(1.);
    } else {
        s = (q * r - w * p) / d;
        t = (-s * r - q) / w;
    }
    if ((ccdIsZero(s) || s > CCD_ZERO) && (ccdEq(s, CCD_ONE) || s < CCD_ONE) && (ccdIsZero(t) || t > CCD_ZERO) &&
        (ccdEq(t, CCD_ONE) || t < CCD_ONE) && (ccdEq(t + s, CCD_ONE) || t + s < CCD_ONE)) {
        if (witness) {
            ccdVec3Scale(&d1, s);
            ccdVec3Scale(&d2, t);
            ccdVec3Copy(witness, x0);
            ccdVec3Add(witness, &d1);
            ccdVec3Add(witness, &d2);
            dist = lx_dist2(witness, P);
        } else {
            dist = s * s * v;
            dist += t * t * w;
            dist += CCD_REAL(2.) * s * t * r;
            dist += CCD_REAL(2.) * s * p;
            dist += CCD_REAL(2.) * t * q;
            dist += u;
        }
    } else {
        dist = lx_seg_dist2(P, x0, B, witness);
        dist2 = lx_seg_dist2(P, x0, C, &witness2);
        if (dist2 < dist) {
            dist = dist2;
            if (witness) ccdVec3Copy(witness, &witness2);
        }
        dist2 = lx_seg_dist2(P, B, C, &witness2);
        if (dist2 < dist) {
            dist = dist2;
            if (witness) ccdVec3Copy(witness, &witness2);
        }
    }
    return dist;
}

/* simplex.h */
static int sx_size(const ccd_simplex_t *s) { return s->last + 1; }
static void sx_add(ccd_simplex_t *s, const ccd_support_t *v) { ++s->last; s->ps[s->last] = *v; }
static void sx_set(ccd_simplex_t *s, int pos, const ccd_support_t *a) { s->ps[pos] = *a; }
static void sx_set_size(ccd_simplex_t *s, int size) { s->last = size - 1; }

static void lx_triple_cross(const ccd_vec3_t *a, const ccd_vec3_t *b, const ccd_vec3_t *c, ccd_vec3_t *d) {
    ccd_vec3_t e;
    ccdVec3Cross(&e, a, b);
    ccdVec3Cross(d, &e, c);
}

static int lx_sign(ccd_real_t val) {
    if (ccdIsZero(val)) return 0;
    if (val < CCD_ZERO) return -1;
    return 1;
}

static int lx_abs_lt_eps2(ccd_real_t val) { return CCD_FABS(val) < CCD_EPS * CCD_EPS; } /* isAbsValueLessThanEpsSquared */

/* are_coincident: per axis |p_i - q_i| <= eps max(1, |p_i|, |q_i|) */
static int lx_coincident(const ccd_vec3_t *p, const ccd_vec3_t *q) {
    for (int i = 0; i < 3; ++i) {
        ccd_real_t m = CCD_ONE;
        if (CCD_FABS(p->v[i]) > m) m = CCD_FABS(p->v[i]);
        if (CCD_FABS(q->v[i]) > m) m = CCD_FABS(q->v[i]);
        if (CCD_FABS(p->v[i] - q->v[i]) > m * CCD_EPS) return 0;
    }
    return 1;
}

/* triangle_area_is_zero */
static int lx_tri_area_zero(const ccd_vec3_t *a, const ccd_vec3_t *b, const ccd_vec3_t *c) {
    if (lx_coincident(a, b) || lx_coincident(a, c) || lx_coincident(b, c)) return 1;
    ccd_vec3_t AB, AC, n;
    ccdVec3Sub2(&AB, b, a);
    ccdVec3Sub2(&AC, c, a);
    ccdVec3Normalize(&AB);
    ccdVec3Normalize(&AC);
    ccdVec3Cross(&n, &AB, &AC);
    return CCD_FABS(n.v[0]) < CCD_EPS && CCD_FABS(n.v[1]) < CCD_EPS && CCD_FABS(n.v[2]) < CCD_EPS;
}

static int lx_do_simplex2(ccd_simplex_t *simplex, ccd_vec3_t *dir) {
    const ccd_support_t *A = &simplex->ps[simplex->last], *B = &simplex->ps[0];
    ccd_vec3_t AB, AO, n;
    ccdVec3Sub2(&AB, &B->v, &A->v);
    ccdVec3Copy(&AO, &A->v);
    ccdVec3Scale(&AO, -CCD_ONE);
    ccdVec3Cross(&n, &AB, &AO);
    if (ccdVec3Len2(&n) <= CCD_EPS * CCD_EPS * ccdVec3Len2(&AB) * ccdVec3Len2(&AO)) return 1;
    ccdVec3Cross(dir, &n, &AB); /* tripleCross(AB, AO, AB) */
    return 0;
}

static int lx_do_simplex3(ccd_simplex_t *simplex, ccd_vec3_t *dir) {
    const ccd_support_t *A = &simplex->ps[simplex->last], *B = &simplex->ps[1], *C = &simplex->ps[0];
    ccd_vec3_t AO, AB, AC, ABC, tmp, proj;
    ccd_real_t dot;
    /* touching contact; FCL asks for the projection (libccd issue 55) */
    const ccd_real_t dist2 = lx_tri_dist2(&ccd_vec3_origin, &A->v, &B->v, &C->v, &proj);
    if (lx_abs_lt_eps2(dist2)) return 1;
    if (lx_tri_area_zero(&A->v, &B->v, &C->v)) return -1;
    ccdVec3Copy(&AO, &A->v);
    ccdVec3Scale(&AO, -CCD_ONE);
    ccdVec3Sub2(&AB, &B->v, &A->v);
    ccdVec3Sub2(&AC, &C->v, &A->v);
    ccdVec3Cross(&ABC, &AB, &AC);
    ccdVec3Cross(&tmp, &ABC, &AC);
    dot = ccdVec3Dot(&tmp, &AO);
    int region45 = 0;
    if (ccdIsZero(dot) || dot > CCD_ZERO) {
        dot = ccdVec3Dot(&AC, &AO);
        if (ccdIsZero(dot) || dot > CCD_ZERO) {
            sx_set(simplex, 1, A);
            sx_set_size(simplex, 2);
            lx_triple_cross(&AC, &AO, &AC, dir);
        } else {
            region45 = 1;
        }
    } else {
        ccdVec3Cross(&tmp, &AB, &ABC);
        dot = ccdVec3Dot(&tmp, &AO);
        if (ccdIsZero(dot) || dot > CCD_ZERO) {
            region45 = 1;
        } else {
            dot = ccdVec3Dot(&ABC, &AO);
            if (ccdIsZero(dot) || dot > CCD_ZERO) {
                ccdVec3Copy(dir, &ABC);
            } else {
                ccd_support_t Ctmp = *C;
                sx_set(simplex, 0, B);
                sx_set(simplex, 1, &Ctmp);
                ccdVec3Copy(dir, &ABC);
                ccdVec3Scale(dir, -CCD_ONE);
            }
        }
    }
    if (region45) { /* ccd_do_simplex3_45 */
        dot = ccdVec3Dot(&AB, &AO);
        if (ccdIsZero(dot) || dot > CCD_ZERO) {
            sx_set(simplex, 0, B);
            sx_set(simplex, 1, A);
            sx_set_size(simplex, 2);
            lx_triple_cross(&AB, &AO, &AB, dir);
        } else {
            sx_set(simplex, 0, A);
            sx_set_size(simplex, 1);
            ccdVec3Copy(dir, &AO);
        }
    }
    return 0;
}

static int lx_do_simplex4(ccd_simplex_t *simplex, ccd_vec3_t *dir) {
    const ccd_support_t *A = &simplex->ps[simplex->last], *B = &simplex->ps[2], *C = &simplex->ps[1],
                        *D = &simplex->ps[0];
    ccd_vec3_t AO, AB, AC, AD, ABC, ACD, ADB;
    int B_on_ACD, C_on_ADB, D_on_ABC, AB_O, AC_O, AD_O;
    ccd_real_t dist;
    dist = lx_tri_dist2(&A->v, &B->v, &C->v, &D->v, NULL);
    if (lx_abs_lt_eps2(dist)) return -1;
    dist = lx_tri_dist2(&ccd_vec3_origin, &A->v, &B->v, &C->v, NULL);
    if (lx_abs_lt_eps2(dist)) return 1;
    dist = lx_tri_dist2(&ccd_vec3_origin, &A->v, &C->v, &D->v, NULL);
    if (lx_abs_lt_eps2(dist)) return 1;
    dist = lx_tri_dist2(&ccd_vec3_origin, &A->v, &B->v, &D->v, NULL);
    if (lx_abs_lt_eps2(dist)) return 1;
    dist = lx_tri_dist2(&ccd_vec3_origin, &B->v, &C->v, &D->v, NULL);
    if (lx_abs_lt_eps2(dist)) return 1;
    ccdVec3Copy(&AO, &A->v);
    ccdVec3Scale(&AO, -CCD_ONE);
    ccdVec3Sub2(&AB, &B->v, &A->v);
    ccdVec3Sub2(&AC, &C->v, &A->v);
    ccdVec3Sub2(&AD, &D->v, &A->v);
    ccdVec3Cross(&ABC, &AB, &AC);
    ccdVec3Cross(&ACD, &AC, &AD);
    ccdVec3Cross(&ADB, &AD, &AB);
    B_on_ACD = lx_sign(ccdVec3Dot(&ACD, &AB));
    C_on_ADB = lx_sign(ccdVec3Dot(&ADB, &AC));
    D_on_ABC = lx_sign(ccdVec3Dot(&ABC, &AD));
    AB_O = lx_sign(ccdVec3Dot(&ACD, &AO)) == B_on_ACD;
    AC_O = lx_sign(ccdVec3Dot(&ADB, &AO)) == C_on_ADB;
    AD_O = lx_sign(ccdVec3Dot(&ABC, &AO)) == D_on_ABC;
    if (AB_O && AC_O && AD_O) return 1;
    if (!AB_O) {
        sx_set(simplex, 2, A);
        sx_set_size(simplex, 3);
    } else if (!AC_O) {
        sx_set(simplex, 1, D);
        sx_set(simplex, 0, B);
        sx_set(simplex, 2, A);
        sx_set_size(simplex, 3);
    } else {
        sx_set(simplex, 0, C);
        sx_set(simplex, 1, B);
        sx_set(simplex, 2, A);
        sx_set_size(simplex, 3);
    }
    return lx_do_simplex3(simplex, dir);
}

static int lx_do_simplex(ccd_simplex_t *simplex, ccd_vec3_t *dir) {
    const int n = sx_size(simplex);
    if (n == 2) return lx_do_simplex2(simplex, dir);
    if (n == 3) return lx_do_simplex3(simplex, dir);
    return lx_do_simplex4(simplex, dir);
}

/* __ccdGJK: 0 = intersection found, -1 = not (the simplex is left for _ccdDist) */
static int lx_gjk(const gjk_obj *o1, const gjk_obj *o2, ccd_simplex_t *simplex) {
    ccd_vec3_t dir;
    ccd_support_t last;
    simplex->last = -1;
    ccdVec3Set(&dir, CCD_ONE, CCD_ZERO, CCD_ZERO); /* ccdFirstDirDefault */
    ccd_support(o1, o2, &dir, &last);
    sx_add(simplex, &last);
    ccdVec3Copy(&dir, &last.v);
    ccdVec3Scale(&dir, -CCD_ONE);
    for (unsigned long it = 0; it < LX_MAX_ITER; ++it) {
        ccd_support(o1, o2, &dir, &last);
        if (ccdVec3Dot(&last.v, &dir) < CCD_ZERO) return -1;
        sx_add(simplex, &last);
        const int r = lx_do_simplex(simplex, &dir);
        if (r == 1) return 0;
        if (r == -1) return -1;
        if (ccdIsZero(ccdVec3Len2(&dir))) return -1;
    }
    return -1;
}

/* simplexReduceToTriangle */
static ccd_real_t lx_reduce_to_triangle(ccd_simplex_t *simplex, ccd_real_t dist, ccd_vec3_t *best_witness) {
    ccd_real_t newdist;
    ccd_vec3_t witness;
    int best = -1;
    for (int i = 0; i < 3; ++i) {
        newdist = lx_tri_dist2(&ccd_vec3_origin, &simplex->ps[i == 0 ? 3 : 0].v, &simplex->ps[i == 1 ? 3 : 1].v,
                               &simplex->ps[i == 2 ? 3 : 2].v, &witness);
        newdist = CCD_SQRT(newdist);
        if (newdist < dist) {
            dist = newdist;
            best = i;
            ccdVec3Copy(best_witness, &witness);
        }
    }
    if (best >= 0) sx_set(simplex, best, &simplex->ps[3]);
    sx_set_size(simplex, 3);
    return dist;
}

/* extractObjectPointsFromPoint / FromSegment / extractClosestPoints */
static void lx_points_from_point(const ccd_support_t *q, ccd_vec3_t *p1, ccd_vec3_t *p2) {
    *p1 = q->v1;
    *p2 = q->v2;
}

static void lx_lerp(const ccd_vec3_t *a, const ccd_vec3_t *b, ccd_real_t s, ccd_vec3_t *p) {
    ccd_vec3_t sAB;
    ccdVec3Sub2(&sAB, b, a);
    ccdVec3Scale(&sAB, s);
    ccdVec3Copy(p, a);
    ccdVec3Add(p, &sAB);
}

static void lx_points_from_segment(const ccd_support_t *a, const ccd_support_t *b, ccd_vec3_t *p1, ccd_vec3_t *p2,
                                   const ccd_vec3_t *p) {
    ccd_vec3_t AB;
    ccdVec3Sub2(&AB, &b->v, &a->v);
    const ccd_real_t ax = CCD_FABS(AB.v[0]), ay = CCD_FABS(AB.v[1]), az = CCD_FABS(AB.v[2]);
    ccd_real_t A_i, AB_i, p_i;
    if (ax >= ay && ax >= az) {
        A_i = a->v.v[0]; AB_i = AB.v[0]; p_i = p->v[0];
    } else if (ay >= az) {
        A_i = a->v.v[1]; AB_i = AB.v[1]; p_i = p->v[1];
    } else {
        A_i = a->v.v[2]; AB_i = AB.v[2]; p_i = p->v[2];
    }
    if (CCD_FABS(AB_i) < CCD_EPS) {
        lx_points_from_point(a, p1, p2);
        return;
    }
    const ccd_real_t s = (p_i - A_i) / AB_i;
    lx_lerp(&a->v1, &b->v1, s, p1);
    lx_lerp(&a->v2, &b->v2, s, p2);
}

static void lx_extract_closest(const ccd_simplex_t *simplex, ccd_vec3_t *p1, ccd_vec3_t *p2, const ccd_vec3_t *p) {
    const int n = sx_size(simplex);
    const ccd_support_t *ps = simplex->ps;
    if (n == 1) {
        lx_points_from_point(&ps[0], p1, p2);
        return;
    }
    if (n == 2) {
        lx_points_from_segment(&ps[0], &ps[1], p1, p2, p);
        return;
    }
    if (lx_tri_area_zero(&ps[0].v, &ps[1].v, &ps[2].v)) {
        ccd_vec3_t AB, AC, BC;
        ccdVec3Sub2(&AB, &ps[1].v, &ps[0].v);
        ccdVec3Sub2(&AC, &ps[2].v, &ps[0].v);
        ccdVec3Sub2(&BC, &ps[2].v, &ps[1].v);
        const ccd_real_t ab = ccdVec3Len2(&AB), ac = ccdVec3Len2(&AC), bc = ccdVec3Len2(&BC);
        int ia, ib;
        if (ab >= ac && ab >= bc) { ia = 0; ib = 1; }
        else if (ac >= ab && ac >= bc) { ia = 0; ib = 2; }
        else { ia = 1; ib = 2; }
        lx_points_from_segment(&ps[ia], &ps[ib], p1, p2, p);
        return;
    }
    ccd_vec3_t r_AB, r_AC, nrm, r_Ap, c1, c2;
    ccdVec3Sub2(&r_AB, &ps[1].v, &ps[0].v);
    ccdVec3Sub2(&r_AC, &ps[2].v, &ps[0].v);
    ccdVec3Cross(&nrm, &r_AB, &r_AC);
    const ccd_real_t nn = ccdVec3Len2(&nrm);
    ccdVec3Sub2(&r_Ap, p, &ps[0].v);
    ccdVec3Cross(&c1, &r_Ap, &r_AC);
    ccdVec3Cross(&c2, &r_AB, &r_Ap);
    const ccd_real_t beta = ccdVec3Dot(&nrm, &c1) / nn;
    const ccd_real_t gamma = ccdVec3Dot(&nrm, &c2) / nn;
    for (int side = 0; side < 2; ++side) {
        const ccd_vec3_t *A = side ? &ps[0].v2 : &ps[0].v1, *B = side ? &ps[1].v2 : &ps[1].v1,
                         *C = side ? &ps[2].v2 : &ps[2].v1;
        ccd_vec3_t *out = side ? p2 : p1, t;
        ccdVec3Copy(out, A);
        ccdVec3Sub2(&t, B, A);
        ccdVec3Scale(&t, beta);
        ccdVec3Add(out, &t);
        ccdVec3Sub2(&t, C, A);
        ccdVec3Scale(&t, gamma);
        ccdVec3Add(out, &t);
    }
}

/* _ccdDist: GJK distance iteration from the simplex __ccdGJK left */
static ccd_real_t lx_dist(const gjk_obj *o1, const gjk_obj *o2, ccd_real_t dist_tol, ccd_simplex_t *simplex,
                          ccd_vec3_t *p1, ccd_vec3_t *p2) {
    ccd_support_t last;
    ccd_vec3_t dir;
    ccd_real_t dist, last_dist = CCD_REAL_MAX;
    for (unsigned long it = 0; it < LX_MAX_ITER; ++it) {
        const int n = sx_size(simplex);
        if (n == 1) {
            ccdVec3Copy(&dir, &simplex->ps[0].v);
            dist = ccdVec3Len2(&simplex->ps[0].v);
            dist = CCD_SQRT(dist);
        } else if (n == 2) {
            dist = lx_seg_dist2(&ccd_vec3_origin, &simplex->ps[0].v, &simplex->ps[1].v, &dir);
            dist = CCD_SQRT(dist);
        } else if (n == 3) {
            dist = lx_tri_dist2(&ccd_vec3_origin, &simplex->ps[0].v, &simplex->ps[1].v, &simplex->ps[2].v, &dir);
            dist = CCD_SQRT(dist);
        } else {
            dist = lx_reduce_to_triangle(simplex, last_dist, &dir);
        }
        if (ccdIsZero(dist)) return -CCD_ONE; /* touching */
        if ((last_dist - dist) < dist_tol) {
            lx_extract_closest(simplex, p1, p2, &dir);
            return dist;
        }
        ccd_vec3_t sdir = dir; /* the witness stays in dir (see the header) */
        ccdVec3Scale(&sdir, -CCD_ONE);
        ccdVec3Normalize(&sdir);
        ccd_support(o1, o2, &sdir, &last);
        last_dist = dist;
        dist = ccdVec3Len2(&last.v);
        dist = CCD_SQRT(dist);
        if (CCD_FABS(last_dist - dist) < dist_tol) { /* no progress: the support pair itself */
            *p1 = last.v1;
            *p2 = last.v2;
            return last_dist;
        }
        sx_add(simplex, &last);
    }
    return -CCD_REAL(1.);
}

/* ccdGJKDist2 */
static ccd_real_t lx_gjk_dist2(const gjk_obj *o1, const gjk_obj *o2, ccd_real_t dist_tol, ccd_vec3_t *p1,
                               ccd_vec3_t *p2) {
    ccd_simplex_t simplex;
    if (lx_gjk(o1, o2, &simplex) == 0) return -CCD_ONE;
    return lx_dist(o1, o2, dist_tol, &simplex, p1, p2);
}

/* ------------------------------------------------- polytope (libccd 2.1) */
typedef struct lx_el lx_el;
struct lx_el {
    int type;
    ccd_real_t dist;
    ccd_vec3_t witness;
    ccd_support_t v;   /* vertex */
    lx_el *vtx[2];     /* edge: vertex[0..1] */
    lx_el *fc[2];      /* edge: faces[0..1] (aligned to the lower index) */
    lx_el *ed[3];      /* face: edge[0..2] */
    lx_el *new_edge;   /* vertex: expandPolytope's map_vertex_to_new_edge */
    int mark;          /* face: visible; edge: 1 internal, 2 border */
};
typedef struct {
    lx_el **a;
    int n, cap;
} lx_list;
typedef struct {
    lx_list v, e, f;
    lx_el *nearest;
    ccd_real_t nearest_dist;
    int nearest_type;
} lx_pt;

static void lx_list_push(lx_list *l, lx_el *x) {
    if (l->n == l->cap) {
        l->cap = l->cap ? 2 * l->cap : 64;
        l->a = realloc(l->a, sizeof(lx_el *) * (size_t)l->cap);
    }
    l->a[l->n++] = x;
}
static void lx_list_del(lx_list *l, lx_el *x) { /* ccdListDel: the others keep their order */
    for (int i = 0; i < l->n; ++i)
        if (l->a[i] == x) {
            memmove(l->a + i, l->a + i + 1, sizeof(lx_el *) * (size_t)(l->n - i - 1));
            --l->n;
            return;
        }
}

static void lx_pt_init(lx_pt *pt) {
    memset(pt, 0, sizeof *pt);
    pt->nearest = NULL;
    pt->nearest_dist = CCD_REAL_MAX;
    pt->nearest_type = 3;
}
static void lx_pt_destroy(lx_pt *pt) {
    lx_list *ls[3] = {&pt->v, &pt->e, &pt->f};
    for (int k = 0; k < 3; ++k) {
        for (int i = 0; i < ls[k]->n; ++i) free(ls[k]->a[i]);
        free(ls[k]->a);
    }
}

/* _ccdPtNearestUpdate */
static void lx_nearest_update(lx_pt *pt, lx_el *el) {
    if (ccdEq(pt->nearest_dist, el->dist)) {
        if (el->type < pt->nearest_type) {
            pt->nearest = el;
            pt->nearest_dist = el->dist;
            pt->nearest_type = el->type;
        }
    } else if (el->dist < pt->nearest_dist) {
        pt->nearest = el;
        pt->nearest_dist = el->dist;
        pt->nearest_type = el->type;
    }
}
/* ccdPtNearest (_ccdPtNearestRenew: vertices, then edges, then faces) */
static lx_el *lx_pt_nearest(lx_pt *pt) {
    if (!pt->nearest) {
        pt->nearest_dist = CCD_REAL_MAX;
        pt->nearest_type = 3;
        pt->nearest = NULL;
        for (int i = 0; i < pt->v.n; ++i) lx_nearest_update(pt, pt->v.a[i]);
        for (int i = 0; i < pt->e.n; ++i) lx_nearest_update(pt, pt->e.a[i]);
        for (int i = 0; i < pt->f.n; ++i) lx_nearest_update(pt, pt->f.a[i]);
    }
    return pt->nearest;
}

static lx_el *lx_add_vertex(lx_pt *pt, const ccd_support_t *v) {
    lx_el *x = calloc(1, sizeof *x);
    x->type = CCD_PT_VERTEX;
    x->v = *v;
    x->dist = ccdVec3Len2(&x->v.v);
    ccdVec3Copy(&x->witness, &x->v.v);
    lx_list_push(&pt->v, x);
    lx_nearest_update(pt, x);
    return x;
}
static lx_el *lx_add_edge(lx_pt *pt, lx_el *v1, lx_el *v2) {
    lx_el *x = calloc(1, sizeof *x);
    x->type = CCD_PT_EDGE;
    x->vtx[0] = v1;
    x->vtx[1] = v2;
    x->dist = lx_seg_dist2(&ccd_vec3_origin, &v1->v.v, &v2->v.v, &x->witness);
    lx_list_push(&pt->e, x);
    lx_nearest_update(pt, x);
    return x;
}
static void lx_face_vertices(const lx_el *f, lx_el *out[3]) { /* ccdPtFaceVec3 / getFaceVertices order */
    out[0] = f->ed[0]->vtx[0];
    out[1] = f->ed[0]->vtx[1];
    out[2] = (f->ed[1]->vtx[0] != out[0] && f->ed[1]->vtx[0] != out[1]) ? f->ed[1]->vtx[0] : f->ed[1]->vtx[1];
}
static lx_el *lx_add_face(lx_pt *pt, lx_el *e1, lx_el *e2, lx_el *e3) {
    lx_el *x = calloc(1, sizeof *x), *vs[3];
    x->type = CCD_PT_FACE;
    x->ed[0] = e1;
    x->ed[1] = e2;
    x->ed[2] = e3;
    lx_face_vertices(x, vs);
    x->dist = lx_tri_dist2(&ccd_vec3_origin, &vs[0]->v.v, &vs[1]->v.v, &vs[2]->v.v, &x->witness);
    for (int i = 0; i < 3; ++i) {
        if (x->ed[i]->fc[0] == NULL) x->ed[i]->fc[0] = x;
        else x->ed[i]->fc[1] = x;
    }
    lx_list_push(&pt->f, x);
    lx_nearest_update(pt, x);
    return x;
}
static void lx_del_face(lx_pt *pt, lx_el *f) {
    for (int i = 0; i < 3; ++i) {
        lx_el *e = f->ed[i];
        if (e->fc[0] == f) e->fc[0] = e->fc[1];
        e->fc[1] = NULL;
    }
    lx_list_del(&pt->f, f);
    if (pt->nearest == f) pt->nearest = NULL;
    free(f);
}
static void lx_del_edge(lx_pt *pt, lx_el *e) {
    lx_list_del(&pt->e, e);
    if (pt->nearest == e) pt->nearest = NULL;
    free(e);
}

/* simplexToPolytope4 (libccd 2.1; the a..d pointers alias the simplex, which
 * the degeneracy checks rewrite in place) */
static int lx_to_polytope3(const gjk_obj *o1, const gjk_obj *o2, const ccd_simplex_t *simplex, lx_pt *pt,
                           lx_el **nearest);
static int lx_to_polytope4(const gjk_obj *o1, const gjk_obj *o2, ccd_simplex_t *simplex, lx_pt *pt, lx_el **nearest) {
    const ccd_support_t *a = &simplex->ps[0], *b = &simplex->ps[1], *c = &simplex->ps[2], *d = &simplex->ps[3];
    int use3 = 0;
    ccd_real_t dist = lx_tri_dist2(&a->v, &b->v, &c->v, &d->v, NULL);
    if (ccdIsZero(dist)) use3 = 1;
    dist = lx_tri_dist2(&a->v, &c->v, &d->v, &b->v, NULL);
    if (ccdIsZero(dist)) {
        use3 = 1;
        sx_set(simplex, 1, c);
        sx_set(simplex, 2, d);
    }
    dist = lx_tri_dist2(&a->v, &b->v, &d->v, &c->v, NULL);
    if (ccdIsZero(dist)) {
        use3 = 1;
        sx_set(simplex, 2, d);
    }
    dist = lx_tri_dist2(&b->v, &c->v, &d->v, &a->v, NULL);
    if (ccdIsZero(dist)) {
        use3 = 1;
        sx_set(simplex, 0, b);
        sx_set(simplex, 1, c);
        sx_set(simplex, 2, d);
    }
    if (use3) {
        sx_set_size(simplex, 3);
        return lx_to_polytope3(o1, o2, simplex, pt, nearest);
    }
    lx_el *v[4], *e[6];
    for (int i = 0; i < 4; ++i) v[i] = lx_add_vertex(pt, &simplex->ps[i]);
    e[0] = lx_add_edge(pt, v[0], v[1]);
    e[1] = lx_add_edge(pt, v[1], v[2]);
    e[2] = lx_add_edge(pt, v[2], v[0]);
    e[3] = lx_add_edge(pt, v[3], v[0]);
    e[4] = lx_add_edge(pt, v[3], v[1]);
    e[5] = lx_add_edge(pt, v[3], v[2]);
    lx_add_face(pt, e[0], e[1], e[2]);
    lx_add_face(pt, e[3], e[4], e[0]);
    lx_add_face(pt, e[4], e[5], e[1]);
    lx_add_face(pt, e[5], e[3], e[2]);
    return 0;
}

/* simplexToPolytope3: -1 = touching contact (*nearest = the triangle) */
static int lx_to_polytope3(const gjk_obj *o1, const gjk_obj *o2, const ccd_simplex_t *simplex, lx_pt *pt,
                           lx_el **nearest) {
    const ccd_support_t *a = &simplex->ps[0], *b = &simplex->ps[1], *c = &simplex->ps[2];
    ccd_support_t d, d2;
    ccd_vec3_t ab, ac, dir;
    lx_el *v[5], *e[9];
    *nearest = NULL;
    ccdVec3Sub2(&ab, &b->v, &a->v);
    ccdVec3Sub2(&ac, &c->v, &a->v);
    ccdVec3Cross(&dir, &ab, &ac);
    ccd_support(o1, o2, &dir, &d);
    const ccd_real_t dist = lx_tri_dist2(&d.v, &a->v, &b->v, &c->v, NULL);
    ccdVec3Scale(&dir, -CCD_ONE);
    ccd_support(o1, o2, &dir, &d2);
    const ccd_real_t dist2 = lx_tri_dist2(&d2.v, &a->v, &b->v, &c->v, NULL);
    if (ccdIsZero(dist) || ccdIsZero(dist2)) {
        v[0] = lx_add_vertex(pt, a);
        v[1] = lx_add_vertex(pt, b);
        v[2] = lx_add_vertex(pt, c);
        e[0] = lx_add_edge(pt, v[0], v[1]);
        e[1] = lx_add_edge(pt, v[1], v[2]);
        e[2] = lx_add_edge(pt, v[2], v[0]);
        *nearest = lx_add_face(pt, e[0], e[1], e[2]);
        return -1;
    }
    v[0] = lx_add_vertex(pt, a);
    v[1] = lx_add_vertex(pt, b);
    v[2] = lx_add_vertex(pt, c);
    v[3] = lx_add_vertex(pt, &d);
    v[4] = lx_add_vertex(pt, &d2);
    e[0] = lx_add_edge(pt, v[0], v[1]);
    e[1] = lx_add_edge(pt, v[1], v[2]);
    e[2] = lx_add_edge(pt, v[2], v[0]);
    e[3] = lx_add_edge(pt, v[3], v[0]);
    e[4] = lx_add_edge(pt, v[3], v[1]);
    e[5] = lx_add_edge(pt, v[3], v[2]);
    e[6] = lx_add_edge(pt, v[4], v[0]);
    e[7] = lx_add_edge(pt, v[4], v[1]);
    e[8] = lx_add_edge(pt, v[4], v[2]);
    lx_add_face(pt, e[3], e[4], e[0]);
    lx_add_face(pt, e[4], e[5], e[1]);
    lx_add_face(pt, e[5], e[3], e[2]);
    lx_add_face(pt, e[6], e[7], e[0]);
    lx_add_face(pt, e[7], e[8], e[1]);
    lx_add_face(pt, e[8], e[6], e[2]);
    return 0;
}

/* the 2-simplex (origin on segment AB): 0 and a tetrahedron in *simplex, or
 * -1 (touching: the segment as the polytope, *nearest = its edge) */
static int lx_segment_to_tetrahedron(const gjk_obj *o1, const gjk_obj *o2, ccd_simplex_t *simplex, lx_pt *pt,
                                     lx_el **nearest) {
    const ccd_support_t A = simplex->ps[0], B = simplex->ps[1];
    ccd_vec3_t AB, axis, dir, n, t;
    ccd_support_t s0, s1, s2;
    ccdVec3Sub2(&AB, &B.v, &A.v);
    int k = 0;
    if (CCD_FABS(AB.v[1]) < CCD_FABS(AB.v[k])) k = 1;
    if (CCD_FABS(AB.v[2]) < CCD_FABS(AB.v[k])) k = 2;
    ccdVec3Set(&axis, k == 0 ? CCD_ONE : CCD_ZERO, k == 1 ? CCD_ONE : CCD_ZERO, k == 2 ? CCD_ONE : CCD_ZERO);
    ccdVec3Cross(&dir, &AB, &axis);
    ccd_support(o1, o2, &dir, &s0);
    if (ccdVec3Eq(&s0.v, &A.v) || ccdVec3Eq(&s0.v, &B.v)) {
        ccdVec3Scale(&dir, -CCD_ONE);
        ccd_support(o1, o2, &dir, &s0);
    }
    int touching = ccdVec3Eq(&s0.v, &A.v) || ccdVec3Eq(&s0.v, &B.v);
    if (!touching) {
        ccdVec3Sub2(&t, &s0.v, &A.v);
        ccdVec3Cross(&n, &AB, &t);
        ccd_support(o1, o2, &n, &s1);
        ccdVec3Scale(&n, -CCD_ONE);
        ccd_support(o1, o2, &n, &s2);
        ccdVec3Scale(&n, -CCD_ONE);
        ccd_vec3_t d1, d2;
        ccdVec3Sub2(&d1, &s1.v, &A.v);
        ccdVec3Sub2(&d2, &s2.v, &A.v);
        const ccd_real_t h1 = ccdVec3Dot(&d1, &n), h2 = -ccdVec3Dot(&d2, &n);
        if (ccdIsZero(h1) && ccdIsZero(h2)) touching = 1;
        else {
            simplex->last = -1;
            sx_add(simplex, &A);
            sx_add(simplex, &B);
            sx_add(simplex, &s0);
            sx_add(simplex, h1 >= h2 ? &s1 : &s2);
            return 0;
        }
    }
    lx_el *v0 = lx_add_vertex(pt, &A), *v1 = lx_add_vertex(pt, &B);
    *nearest = lx_add_edge(pt, v0, v1);
    return -1;
}

/* faceNormalPointingOutward (not normalised) */
static ccd_vec3_t lx_face_normal_out(const lx_pt *pt, const lx_el *face) {
    ccd_vec3_t e1, e2, dir, unit_dir;
    ccdVec3Sub2(&e1, &face->ed[0]->vtx[1]->v.v, &face->ed[0]->vtx[0]->v.v);
    ccdVec3Sub2(&e2, &face->ed[1]->vtx[1]->v.v, &face->ed[1]->vtx[0]->v.v);
    ccdVec3Cross(&dir, &e1, &e2);
    const ccd_real_t dir_norm = CCD_SQRT(ccdVec3Len2(&dir));
    unit_dir = dir;
    ccdVec3Scale(&unit_dir, (ccd_real_t)(1.0 / (double)dir_norm));
    const ccd_real_t dist_tol = CCD_REAL(0.01);
    const ccd_vec3_t *f0 = &face->ed[0]->vtx[0]->v.v;
    const ccd_real_t origin_distance_to_plane = ccdVec3Dot(&unit_dir, f0);
    if (origin_distance_to_plane < -dist_tol) {
        ccdVec3Scale(&dir, -CCD_ONE);
    } else if (-dist_tol <= origin_distance_to_plane && origin_distance_to_plane <= dist_tol) {
        ccd_real_t max_d = -CCD_REAL_MAX, min_d = CCD_REAL_MAX;
        for (int i = 0; i < pt->v.n; ++i) {
            ccd_vec3_t diff;
            ccdVec3Sub2(&diff, &pt->v.a[i]->v.v, f0);
            const ccd_real_t d = ccdVec3Dot(&unit_dir, &diff);
            if (d > dist_tol) {
                ccdVec3Scale(&dir, -CCD_ONE);
                return dir;
            } else if (d < -dist_tol) {
                return dir;
            } else {
                if (d > max_d) max_d = d;
                if (d < min_d) min_d = d;
            }
        }
        if (max_d > CCD_FABS(min_d)) ccdVec3Scale(&dir, -CCD_ONE);
    }
    return dir;
}

static int lx_outside_face(const lx_pt *pt, const lx_el *f, const ccd_vec3_t *p) {
    ccd_vec3_t n = lx_face_normal_out(pt, f), r;
    ccdVec3Sub2(&r, p, &f->ed[0]->vtx[0]->v.v);
    return ccdVec3Dot(&n, &r) > CCD_ZERO;
}

typedef struct {
    lx_el **vis, **internal, **border;
    int nv, ni, nb;
} lx_patch;

static void lx_patch_push(lx_el ***a, int *n, lx_el *x) {
    if ((*n & 63) == 0) *a = realloc(*a, sizeof(lx_el *) * (size_t)(*n + 64));
    (*a)[(*n)++] = x;
}

/* computeVisiblePatchRecursive */
static void lx_patch_rec(const lx_pt *pt, lx_el *f, int edge_index, const ccd_vec3_t *q, lx_patch *P) {
    lx_el *edge = f->ed[edge_index];
    lx_el *g = edge->fc[0] == f ? edge->fc[1] : edge->fc[0];
    if (!g->mark) {
        if (lx_outside_face(pt, g, q)) {
            g->mark = 1;
            lx_patch_push(&P->vis, &P->nv, g);
            if (!edge->mark) { edge->mark = 1; lx_patch_push(&P->internal, &P->ni, edge); }
            for (int i = 0; i < 3; ++i)
                if (g->ed[i] != edge) lx_patch_rec(pt, g, i, q, P);
        } else if (!edge->mark) {
            edge->mark = 2;
            lx_patch_push(&P->border, &P->nb, edge);
        }
    } else if (!edge->mark) {
        edge->mark = 1;
        lx_patch_push(&P->internal, &P->ni, edge);
    }
}

/* expandPolytope: 0, or LX_THROW */
static int lx_expand(lx_pt *pt, lx_el *el, const ccd_support_t *newv) {
    lx_el *start = NULL;
    if (el->type == CCD_PT_VERTEX) return LX_THROW;
    if (el->type == CCD_PT_FACE) {
        start = el;
    } else {
        if (lx_outside_face(pt, el->fc[0], &newv->v)) start = el->fc[0];
        else if (lx_outside_face(pt, el->fc[1], &newv->v)) start = el->fc[1];
        else return LX_THROW;
    }
    lx_patch P;
    memset(&P, 0, sizeof P);
    start->mark = 1;
    lx_patch_push(&P.vis, &P.nv, start);
    for (int i = 0; i < 3; ++i) lx_patch_rec(pt, start, i, &newv->v, &P);
    for (int i = 0; i < P.nv; ++i) lx_del_face(pt, P.vis[i]);
    for (int i = 0; i < P.ni; ++i) lx_del_edge(pt, P.internal[i]);
    lx_el *nv = lx_add_vertex(pt, newv);
    for (int i = 0; i < pt->v.n; ++i) pt->v.a[i]->new_edge = NULL;
    for (int b = 0; b < P.nb; ++b) {
        lx_el *be = P.border[b], *e[2];
        be->mark = 0;
        for (int i = 0; i < 2; ++i) {
            if (!be->vtx[i]->new_edge) be->vtx[i]->new_edge = lx_add_edge(pt, nv, be->vtx[i]);
            e[i] = be->vtx[i]->new_edge;
        }
        lx_add_face(pt, be, e[0], e[1]);
    }
    free(P.vis);
    free(P.internal);
    free(P.border);
    return 0;
}

/* supportEPADirection: 0, or LX_THROW */
static int lx_epa_direction(const lx_pt *pt, const lx_el *el, ccd_vec3_t *dir) {
    if (ccdIsZero(el->dist)) {
        if (el->type != CCD_PT_FACE) return LX_THROW;
        *dir = lx_face_normal_out(pt, el);
    } else {
        ccdVec3Copy(dir, &el->witness);
    }
    ccdVec3Normalize(dir);
    return 0;
}

/* nextSupport: 0 = expand, -1 = converged, LX_THROW */
static int lx_next_support(const lx_pt *pt, const gjk_obj *o1, const gjk_obj *o2, const lx_el *el, ccd_support_t *out) {
    if (el->type == CCD_PT_VERTEX) return -1;
    ccd_vec3_t dir;
    if (lx_epa_direction(pt, el, &dir)) return LX_THROW;
    ccd_support(o1, o2, &dir, out);
    const ccd_real_t dist = ccdVec3Dot(&out->v, &dir);
    if (dist - CCD_SQRT(el->dist) < LX_EPA_TOL) return -1;
    ccd_real_t d2;
    if (el->type == CCD_PT_EDGE) {
        d2 = lx_seg_dist2(&out->v, &el->vtx[0]->v.v, &el->vtx[1]->v.v, NULL);
    } else {
        lx_el *vs[3];
        lx_face_vertices(el, vs);
        d2 = lx_tri_dist2(&out->v, &vs[0]->v.v, &vs[1]->v.v, &vs[2]->v.v, NULL);
    }
    if (CCD_SQRT(d2) < LX_EPA_TOL) return -1;
    return 0;
}

/* validateNearestFeatureOfPolytopeBeingEdge: the nearer adjacent face */
static lx_el *lx_validate_edge(lx_pt *pt, int *thrown) {
    const lx_el *edge = pt->nearest;
    const ccd_real_t kEps = CCD_REAL(2.) * CCD_EPS;
    double o2f[2];
    const ccd_real_t v0_dist = CCD_SQRT(ccdVec3Len2(&edge->vtx[0]->v.v));
    const ccd_real_t plane_threshold = kEps * (v0_dist > CCD_ONE ? v0_dist : CCD_ONE);
    for (int i = 0; i < 2; ++i) {
        ccd_vec3_t nrm = lx_face_normal_out(pt, edge->fc[i]);
        ccdVec3Normalize(&nrm);
        o2f[i] = (double)(-ccdVec3Dot(&nrm, &edge->vtx[0]->v.v));
        if (o2f[i] > (double)plane_threshold) {
            *thrown = 1;
            return NULL;
        }
    }
    const int k = o2f[0] > o2f[1] ? 0 : 1;
    pt->nearest = edge->fc[k];
    pt->nearest_dist = (ccd_real_t)(o2f[k] * o2f[k]);
    pt->nearest_type = CCD_PT_FACE;
    return pt->nearest;
}

/* the largest EPA polytope (vertices) and the convexity-guard stops since
 * the last read (single-threaded callers; tests check the device's fixed
 * polytope arrays against the first) */
static int lx_epa_max_nv = 0, lx_epa_guard_stops = 0;
int orc_epa_stats(int *guard_stops) {
    const int m = lx_epa_max_nv;
    if (guard_stops) *guard_stops = lx_epa_guard_stops;
    lx_epa_max_nv = 0;
    lx_epa_guard_stops = 0;
    return m;
}

/* __ccdEPA: 0 (nearest set, or NULL), LX_THROW */
static int lx_epa(const gjk_obj *o1, const gjk_obj *o2, ccd_simplex_t *simplex, lx_pt *pt, lx_el **nearest) {
    ccd_support_t supp;
    int ret;
    *nearest = NULL;
    const int size = sx_size(simplex);
    if (size == 4) {
        ret = lx_to_polytope4(o1, o2, simplex, pt, nearest);
    } else if (size == 3) {
        ret = lx_to_polytope3(o1, o2, simplex, pt, nearest);
    } else {
        ret = lx_segment_to_tetrahedron(o1, o2, simplex, pt, nearest);
        if (ret == 0) ret = lx_to_polytope4(o1, o2, simplex, pt, nearest);
    }
    if (ret == -1) return 0; /* touching contact */
    for (;;) {
        *nearest = lx_pt_nearest(pt);
        if (pt->nearest_type == CCD_PT_EDGE) {
            int thrown = 0;
            *nearest = lx_validate_edge(pt, &thrown);
            if (thrown) return LX_THROW;
        }
        const int r = lx_next_support(pt, o1, o2, *nearest, &supp);
        if (r == LX_THROW) return LX_THROW;
        if (r != 0) break;
        /* convexity guard (not in FCL): a face the new support point does not
         * see would be deleted all the same by expandPolytope (it starts the
         * visible patch there unchecked), the polytope turns non-convex and
         * the loop can revisit the same supports forever; stop instead, at
         * the current nearest face */
        if ((*nearest)->type == CCD_PT_FACE && !lx_outside_face(pt, *nearest, &supp.v)) {
            ++lx_epa_guard_stops;
            break;
        }
        if (lx_expand(pt, *nearest, &supp)) return LX_THROW;
    }
    return 0;
}

/* penEPAPosClosest */
static void lx_pen_epa_pos_closest(const lx_el *nearest, ccd_vec3_t *p1, ccd_vec3_t *p2) {
    if (nearest->type == CCD_PT_VERTEX) {
        ccdVec3Copy(p1, &nearest->v.v1);
        ccdVec3Copy(p2, &nearest->v.v2);
        return;
    }
    ccd_simplex_t s;
    s.last = -1;
    if (nearest->type == CCD_PT_EDGE) {
        sx_add(&s, &nearest->vtx[0]->v);
        sx_add(&s, &nearest->vtx[1]->v);
    } else {
        lx_el *vs[3];
        lx_face_vertices(nearest, vs);
        for (int i = 0; i < 3; ++i) sx_add(&s, &vs[i]->v);
    }
    ccd_vec3_t p;
    ccdVec3Copy(&p, &nearest->witness);
    lx_extract_closest(&s, p1, p2, &p);
}


/* ccdGJKSignedDist: *dist (negative: -depth), points; 0 or LX_THROW */
static int lx_gjk_signed_dist(const gjk_obj *o1, const gjk_obj *o2, ccd_real_t dist_tol, ccd_real_t *dist,
                              ccd_vec3_t *p1, ccd_vec3_t *p2) {
    ccd_simplex_t simplex;
    if (lx_gjk(o1, o2, &simplex) == 0) {
        lx_pt pt;
        lx_el *nearest = NULL;
        lx_pt_init(&pt);
        const int ret = lx_epa(o1, o2, &simplex, &pt, &nearest);
        if (pt.v.n > lx_epa_max_nv) lx_epa_max_nv = pt.v.n; /* single-threaded callers only */
        if (ret == LX_THROW) {
            lx_pt_destroy(&pt);
            return LX_THROW;
        }
        if (ret == 0 && nearest) {
            *dist = -CCD_SQRT(nearest->dist);
            lx_pen_epa_pos_closest(nearest, p1, p2);
        } else {
            *dist = -CCD_ONE;
        }
        lx_pt_destroy(&pt);
        return 0;
    }
    *dist = lx_dist(o1, o2, dist_tol, &simplex, p1, p2);
    return 0;
}

/* GJKDistanceImpl (+ GJKDistance / GJKSignedDistance): FCL initialises the
 * points to zero, converts dist and points to double; returns 0 or LX_THROW */
static int fcl_gjk_distance(const gjk_obj *o1, const gjk_obj *o2, int sgn, double dist_tol, double *res, double *p1,
                            double *p2) {
    ccd_vec3_t q1, q2;
    ccdVec3Set(&q1, CCD_ZERO, CCD_ZERO, CCD_ZERO);
    ccdVec3Set(&q2, CCD_ZERO, CCD_ZERO, CCD_ZERO);
    ccd_real_t d;
    if (sgn) {
        if (lx_gjk_signed_dist(o1, o2, (ccd_real_t)dist_tol, &d, &q1, &q2)) return LX_THROW;
    } else {
        d = lx_gjk_dist2(o1, o2, (ccd_real_t)dist_tol, &q1, &q2);
    }
    for (int i = 0; i < 3; ++i) {
        p1[i] = q1.v[i];
        p2[i] = q2.v[i];
    }
    *res = d;
    return 0;
}

/* ----------------------------------------- closed-form shape distances
 * GJKSolver_libccd::shapeDistance's specialisations (ShapeDistanceLibccdImpl
 * [ext FCL 0.7.0 gjk_solver_libccd-inl.h]), used for DistanceRequest() (the
 * signed request always runs GJKSignedDistance): sphereSphereDistance,
 * sphereCapsuleDistance, sphereBoxDistance, sphereCylinderDistance (and the
 * shape-sphere orders with the points swapped), capsuleCapsuleDistance.
 * fp64 (S = double).  1 if the pair has a closed form. */
static void cf_tf_point(const real *T, const real *p, real *o) {
    for (int i = 0; i < 3; ++i) o[i] = ((T[3 * i] * p[0] + T[3 * i + 1] * p[1]) + T[3 * i + 2] * p[2]) + T[9 + i];
}
static real cf_norm(const real *v) { return sqrt((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]); }

/* sphere_sphere-inl.h: diff = o1 - o2; separated when |diff| > r1 + r2 */
static double cf_sphere_sphere(real r1, const real *T1, real r2, const real *T2, double *p1, double *p2) {
    const real o1[3] = {T1[9], T1[10], T1[11]}, o2[3] = {T2[9], T2[10], T2[11]};
    const real diff[3] = {o1[0] - o2[0], o1[1] - o2[1], o1[2] - o2[2]};
    const real len = cf_norm(diff);
    if (len > r1 + r2) {
        for (int i = 0; i < 3; ++i) {
            p1[i] = o1[i] - diff[i] * (r1 / len);
            p2[i] = o2[i] + diff[i] * (r2 / len);
        }
        return len - (r1 + r2);
    }
    return -1.0;
}

/* sphere_capsule-inl.h: the capsule's segment end points tf2 * (0, 0, +-lz/2),
 * lineSegmentPointClosestToPoint, distance = |s_c - sp| - r1 - r2; <= 0 -> -1 */
static double cf_sphere_capsule(real r1, const real *TS, real r2, real lz, const real *TC, double *p1, double *p2) {
    const real a[3] = {0.0, 0.0, 0.5 * lz}, b[3] = {0.0, 0.0, -0.5 * lz};
    real pos1[3], pos2[3], sp[3];
    cf_tf_point(TC, a, pos1);
    cf_tf_point(TC, b, pos2);
    const real sc[3] = {TS[9], TS[10], TS[11]};
    const real v[3] = {pos2[0] - pos1[0], pos2[1] - pos1[1], pos2[2] - pos1[2]};
    const real w[3] = {sc[0] - pos1[0], sc[1] - pos1[1], sc[2] - pos1[2]};
    const real c1 = (w[0] * v[0] + w[1] * v[1]) + w[2] * v[2];
    const real c2 = (v[0] * v[0] + v[1] * v[1]) + v[2] * v[2];
    if (c1 <= 0) memcpy(sp, pos1, sizeof sp);
    else if (c2 <= c1) memcpy(sp, pos2, sizeof sp);
    else {
        const real bb = c1 / c2;
        for (int i = 0; i < 3; ++i) sp[i] = pos1[i] + v[i] * bb;
    }
    real diff[3] = {sc[0] - sp[0], sc[1] - sp[1], sc[2] - sp[2]};
    const real diffN = cf_norm(diff);
    const real distance = diffN - r1 - r2;
    if (distance <= 0) return -1.0;
    const real n = cf_norm(diff); /* diff.normalize() */
    for (int i = 0; i < 3; ++i) diff[i] /= n;
    for (int i = 0; i < 3; ++i) {
        p1[i] = sc[i] - diff[i] * r1;
        p2[i] = sp[i] + diff[i] * r2;
    }
    return distance;
}

/* sphere_box-inl.h sphereBoxDistance: C in the box frame, nearestPointInBox;
 * separated iff clamped and |N C|^2 > r^2 */
static double cf_sphere_box(real r, const real *TS, const real *side, const real *TB, double *pS, double *pB) {
    real c[3], nq[3];
    centre_in_frame(TS, TB, c);
    int clamped = 0;
    for (int i = 0; i < 3; ++i) {
        const real h = side[i] / 2;
        nq[i] = c[i];
        if (c[i] < -h) { clamped = 1; nq[i] = -h; }
        if (c[i] > h) { clamped = 1; nq[i] = h; }
    }
    if (clamped) {
        const real nc[3] = {c[0] - nq[0], c[1] - nq[1], c[2] - nq[2]};
        const real sq = (nc[0] * nc[0] + nc[1] * nc[1]) + nc[2] * nc[2];
        if (sq > r * r) {
            const real d = sqrt(sq);
            real pSb[3];
            for (int i = 0; i < 3; ++i) pSb[i] = (nc[i] / d) * (d - r) + nq[i];
            cf_tf_point(TB, nq, pB);
            cf_tf_point(TB, pSb, pS);
            return d - r;
        }
    }
    return -1.0;
}

/* sphere_cylinder-inl.h sphereCylinderDistance (nearestPointInCylinder) */
static double cf_sphere_cylinder(real r, const real *TS, real rc, real lz, const real *TC, double *pS, double *pC) {
    real c[3], n[3];
    centre_in_frame(TS, TC, c);
    const real h = lz / 2;
    int clamped = 0;
    n[0] = c[0]; n[1] = c[1]; n[2] = c[2];
    if (c[2] > h) { n[2] = h; clamped = 1; }
    else if (c[2] < -h) { n[2] = -h; clamped = 1; }
    const real rd2 = c[0] * c[0] + c[1] * c[1];
    if (rd2 > rc * rc) {
        const real scale = rc / sqrt(rd2);
        n[0] = c[0] * scale;
        n[1] = c[1] * scale;
        clamped = 1;
    }
    if (clamped) {
        const real nc[3] = {c[0] - n[0], c[1] - n[1], c[2] - n[2]};
        const real sq = (nc[0] * nc[0] + nc[1] * nc[1]) + nc[2] * nc[2];
        if (sq > r * r) {
            const real d = sqrt(sq);
            real pSc[3];
            for (int i = 0; i < 3; ++i) pSc[i] = (nc[i] / d) * (d - r) + n[i];
            cf_tf_point(TC, n, pC);
            cf_tf_point(TC, pSc, pS);
            return d - r;
        }
    }
    return -1.0;
}

static real cf_clamp01(real v) { return v < 0.0 ? 0.0 : (v > 1.0 ? 1.0 : v); }

/* capsule_capsule-inl.h: closestPtSegmentSegment of the centre lines
 * (Ericson 5.1.9, eps_78 = DBL_EPSILON^(7/8)); distance = segment distance -
 * r1 - r2 (negative when they overlap: no -1 here); witness points along
 * the centre-line direction (or, for crossing centre lines, the normal of
 * both segments) */
static double cf_capsule_capsule(real r1, real lz1, const real *T1, real r2, real lz2, const real *T2, double *p1,
                                 double *p2) {
    const real eps = 0x1.6a09e667f3bcdp-46, eps2 = eps * eps; /* constants<double>::eps_78() = pow(DBL_EPSILON, 7/8) */
    real P1[3], Q1[3], P2[3], Q2[3];
    for (int i = 0; i < 3; ++i) {
        const real h1 = (lz1 / 2) * T1[3 * i + 2], h2 = (lz2 / 2) * T2[3 * i + 2];
        P1[i] = T1[9 + i] + h1; Q1[i] = T1[9 + i] - h1;
        P2[i] = T2[9 + i] + h2; Q2[i] = T2[9 + i] - h2;
    }
    real d1[3], d2[3], rr[3];
    for (int i = 0; i < 3; ++i) { d1[i] = Q1[i] - P1[i]; d2[i] = Q2[i] - P2[i]; rr[i] = P1[i] - P2[i]; }
    const real a = (d1[0] * d1[0] + d1[1] * d1[1]) + d1[2] * d1[2];
    const real e = (d2[0] * d2[0] + d2[1] * d2[1]) + d2[2] * d2[2];
    const real f = (d2[0] * rr[0] + d2[1] * rr[1]) + d2[2] * rr[2];
    real s, t;
    if (a <= eps2 && e <= eps2) {
        s = t = 0.0;
    } else if (a <= eps2) {
        s = 0.0;
        t = cf_clamp01(f / e);
    } else {
        const real c = (d1[0] * rr[0] + d1[1] * rr[1]) + d1[2] * rr[2];
        if (e <= eps2) {
            t = 0.0;
            s = cf_clamp01(-c / a);
        } else {
            const real b = (d1[0] * d2[0] + d1[1] * d2[1]) + d1[2] * d2[2];
            const real den0 = a * e - b * b, denom = den0 > 0.0 ? den0 : 0.0;
            s = denom > eps2 ? cf_clamp01((b * f - c * e) / denom) : 0.0;
            t = (b * s + f) / e;
            if (t < 0.0) { t = 0.0; s = cf_clamp01(-c / a); }
            else if (t > 1.0) { t = 1.0; s = cf_clamp01((b - c) / a); }
        }
    }
    real N1[3], N2[3], v[3];
    for (int i = 0; i < 3; ++i) { N1[i] = P1[i] + d1[i] * s; N2[i] = P2[i] + d2[i] * t; v[i] = N2[i] - N1[i]; }
    const real seg = sqrt((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]);
    real vh[3];
    if (seg > eps) {
        for (int i = 0; i < 3; ++i) vh[i] = v[i] / seg;
    } else {
        real n[3] = {d1[1] * d2[2] - d1[2] * d2[1], d1[2] * d2[0] - d1[0] * d2[2], d1[0] * d2[1] - d1[1] * d2[0]};
        real nl = cf_norm(n);
        if (!(nl > eps)) { /* parallel: any direction perpendicular to segment 1 */
            const real ax[3] = {fabs(d1[0]) < fabs(d1[1]) ? 1.0 : 0.0, fabs(d1[0]) < fabs(d1[1]) ? 0.0 : 1.0, 0.0};
            n[0] = d1[1] * ax[2] - d1[2] * ax[1]; n[1] = d1[2] * ax[0] - d1[0] * ax[2]; n[2] = d1[0] * ax[1] - d1[1] * ax[0];
            nl = cf_norm(n);
        }
        for (int i = 0; i < 3; ++i) vh[i] = nl > 0.0 ? n[i] / nl : (i == 2 ? 1.0 : 0.0);
    }
    for (int i = 0; i < 3; ++i) { p1[i] = N1[i] + vh[i] * r1; p2[i] = N2[i] - vh[i] * r2; }
    return seg - r1 - r2;
}

static int cf_shape_distance(int ta, const real *pa, const real *Ta, int tb, const real *pb, const real *Tb, double *d,
                             double *p1, double *p2) {
    if (ta == GEOM_SPHERE && tb == GEOM_SPHERE) *d = cf_sphere_sphere(pa[0], Ta, pb[0], Tb, p1, p2);
    else if (ta == GEOM_SPHERE && tb == GEOM_CAPSULE) *d = cf_sphere_capsule(pa[0], Ta, pb[0], pb[1], Tb, p1, p2);
    else if (ta == GEOM_CAPSULE && tb == GEOM_SPHERE) *d = cf_sphere_capsule(pb[0], Tb, pa[0], pa[1], Ta, p2, p1);
    else if (ta == GEOM_SPHERE && tb == GEOM_BOX) *d = cf_sphere_box(pa[0], Ta, pb, Tb, p1, p2);
    else if (ta == GEOM_BOX && tb == GEOM_SPHERE) *d = cf_sphere_box(pb[0], Tb, pa, Ta, p2, p1);
    else if (ta == GEOM_SPHERE && tb == GEOM_CYLINDER) *d = cf_sphere_cylinder(pa[0], Ta, pb[0], pb[1], Tb, p1, p2);
    else if (ta == GEOM_CYLINDER && tb == GEOM_SPHERE) *d = cf_sphere_cylinder(pb[0], Tb, pa[0], pa[1], Ta, p2, p1);
    else if (ta == GEOM_CAPSULE && tb == GEOM_CAPSULE)
        *d = cf_capsule_capsule(pa[0], pa[1], Ta, pb[0], pb[1], Tb, p1, p2);
    else return 0;
    return 1;
}

/* Project<S>::projectLine / projectTriangle [ext FCL 0.7.0
 * narrowphase/detail/convexity_based_algorithm/... project-inl.h] and
 * sphereTriangleDistance with points (sphere_triangle-inl.h): the closed form
 * FCL uses for (Sphere, triangle) leaves of a mesh-shape distance.  -1 when
 * the sphere reaches the triangle (the with-points overload leaves dist
 * unset there; -1 is the value its point-less overload reports). */
typedef struct { real param[4], sqr_distance; } cf_proj;
static cf_proj cf_project_line(const real *a, const real *b, const real *p) {
    cf_proj r = {{0, 0, 0, 0}, -1.0};
    const real d[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
    const real l = (d[0] * d[0] + d[1] * d[1]) + d[2] * d[2];
    if (l > 0) {
        const real pa[3] = {p[0] - a[0], p[1] - a[1], p[2] - a[2]};
        const real t = (pa[0] * d[0] + pa[1] * d[1]) + pa[2] * d[2];
        r.param[1] = (t >= l) ? 1 : ((t <= 0) ? 0 : (t / l));
        r.param[0] = 1 - r.param[1];
        real v[3];
        if (t >= l) for (int i = 0; i < 3; ++i) v[i] = p[i] - b[i];
        else if (t <= 0) for (int i = 0; i < 3; ++i) v[i] = p[i] - a[i];
        else for (int i = 0; i < 3; ++i) v[i] = (a[i] + d[i] * r.param[1]) - p[i];
        r.sqr_distance = (v[0] * v[0] + v[1] * v[1]) + v[2] * v[2];
    }
    return r;
}
static void cf_cross(real *o, const real *a, const real *b) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}
static cf_proj cf_project_triangle(const real *a, const real *b, const real *c, const real *p) {
    cf_proj r = {{0, 0, 0, 0}, -1.0};
    static const int nexti[3] = {1, 2, 0};
    const real *vt[3] = {a, b, c};
    real dl[3][3], n[3];
    for (int i = 0; i < 3; ++i) { dl[0][i] = a[i] - b[i]; dl[1][i] = b[i] - c[i]; dl[2][i] = c[i] - a[i]; }
    cf_cross(n, dl[0], dl[1]);
    const real l = (n[0] * n[0] + n[1] * n[1]) + n[2] * n[2];
    if (l > 0) {
        real mindist = -1;
        for (int i = 0; i < 3; ++i) {
            real vp[3], dn[3];
            for (int k = 0; k < 3; ++k) vp[k] = vt[i][k] - p[k];
            cf_cross(dn, dl[i], n);
            if ((vp[0] * dn[0] + vp[1] * dn[1]) + vp[2] * dn[2] > 0) {
                const int j = nexti[i];
                const cf_proj rl = cf_project_line(vt[i], vt[j], p);
                if (mindist < 0 || rl.sqr_distance < mindist) {
                    mindist = rl.sqr_distance;
                    r.param[i] = rl.param[0];
                    r.param[j] = rl.param[1];
                    r.param[nexti[j]] = 0;
                }
            }
        }
        if (mindist < 0) {
            const real ap[3] = {a[0] - p[0], a[1] - p[1], a[2] - p[2]};
            const real d = (ap[0] * n[0] + ap[1] * n[1]) + ap[2] * n[2];
            const real s = sqrt(l);
            real pp[3], t1[3], t2[3], x[3];
            for (int k = 0; k < 3; ++k) pp[k] = n[k] * (d / l);
            mindist = (pp[0] * pp[0] + pp[1] * pp[1]) + pp[2] * pp[2];
            for (int k = 0; k < 3; ++k) t1[k] = (b[k] - p[k]) - pp[k];
            cf_cross(x, dl[1], t1);
            r.param[0] = cf_norm(x) / s;
            for (int k = 0; k < 3; ++k) t2[k] = (c[k] - p[k]) - pp[k];
            cf_cross(x, dl[2], t2);
            r.param[1] = cf_norm(x) / s;
            r.param[2] = 1 - r.param[0] - r.param[1];
        }
        r.sqr_distance = mindist;
    }
    return r;
}
/* P[0..2]: the triangle in the world frame (tf_mesh * P_i) */
static double cf_sphere_triangle(real radius, const real *TS, const real *P1, const real *P2, const real *P3,
                                 double *pS, double *pT) {
    const real o[3] = {TS[9], TS[10], TS[11]};
    const cf_proj r = cf_project_triangle(P1, P2, P3, o);
    if (r.sqr_distance > radius * radius) {
        real pp[3], dir[3];
        for (int k = 0; k < 3; ++k) pp[k] = (P1[k] * r.param[0] + P2[k] * r.param[1]) + P3[k] * r.param[2];
        for (int k = 0; k < 3; ++k) dir[k] = o[k] - pp[k];
        const real n = cf_norm(dir);
        for (int k = 0; k < 3; ++k) dir[k] /= n;
        for (int k = 0; k < 3; ++k) { pS[k] = o[k] - dir[k] * radius; pT[k] = pp[k]; }
        return sqrt(r.sqr_distance) - radius;
    }
    return -1.0;
}
