/*
 * mpgpu.h -- C ABI of the MI355X batched state-validity checker.
 *
 * This is the drop-in boundary beneath MPlib's PlanningWorld::collide() /
 * collideFull() and the OMPL isStateValid() inner loop.  Plain C, plain
 * pointers and sizes, no C++ or torch types; every call returns an int
 * status (0 = ok) and never throws.  The text of the last error on the
 * calling thread is available from mpg_last_error().
 *
 * Reference interfaces replaced (KolinGuo/MPlib 0.1.1, paths relative to the
 * reference root):
 *   mpg_world_create     <- the mutable FCL/pinocchio state that
 *                           PlanningWorldTpl (src/planning_world.h:52-312),
 *                           ArticulatedModelTpl (src/articulated_model.cpp:15-36),
 *                           FCLModelTpl::init (src/fcl_model.cpp:268-294) and
 *                           AllowedCollisionMatrix (src/collision_matrix.h) hold,
 *                           frozen into an immutable device snapshot.
 *   mpg_collide_batch    <- N x { PlanningWorldTpl::setQposAll(q)
 *                                 (src/planning_world.cpp:250-262);
 *                                 PlanningWorldTpl::collideFull(CollisionRequest())
 *                                 (src/planning_world.cpp:484-490) }
 *                           flags[i]  == collide() (src/planning_world.h:248-250)
 *                           pair_mask == which pairs collideFull() reports,
 *                           after filterCollisions (src/planning_world.cpp:265-274).
 *                           Also the OMPL ValidityCheckerTpl::isValid batch
 *                           (src/ompl_planner.h:59-62): valid = !flags[i].
 *   mpg_fk_batch         <- N x { PinocchioModelTpl::computeForwardKinematics
 *                                 (src/pinocchio_model.cpp:272-274);
 *                                 getLinkPose(i) for every user link
 *                                 (src/pinocchio_model.cpp:277-312) }
 *   mpg_world_destroy    <- shared_ptr release of the above.
 *
 * Memory: buffers are caller-owned.  With MPG_MEM_DEVICE every pointer is a
 * device pointer on the world's device and the work is enqueued on `stream`
 * (a hipStream_t, NULL = default stream) without synchronising.  With
 * MPG_MEM_HOST the call copies through internal device staging buffers and
 * returns after the results are back on the host; batches above the latency
 * path's size (mpg_set_small_batch_max) run as chunks through a pinned ring:
 * the input of one chunk crosses PCIe while earlier chunks compute and are
 * unpacked (internal threads and streams; the call is still synchronous).
 *
 * Threading: a world is immutable after creation; concurrent calls on one
 * world from several host threads are allowed when each uses its own stream
 * and MPG_MEM_DEVICE.  MPG_MEM_HOST calls on one world are serialised.
 * mpg_distance_batch* and mpg_check_motion_batch use scratch owned by the
 * world: their MPG_MEM_DEVICE calls from several streams are ordered on the
 * device (each waits for the previous call's work), never overlapped.
 */
#ifndef MPGPU_H
#define MPGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MPG_VERSION_MAJOR 0
#define MPG_VERSION_MINOR 1

/* status codes */
#define MPG_OK 0
#define MPG_E_INVALID 1     /* bad argument / descriptor                    */
#define MPG_E_UNSUPPORTED 2 /* request or geometry pair not implemented     */
#define MPG_E_HIP 3         /* HIP runtime error                            */
#define MPG_E_NOMEM 4
#define MPG_E_FAILED 5      /* the reference itself fails on this input
                               (FCL throws: mpg_distance_batch_req)      */

/* memory kinds for the batch calls */
#define MPG_MEM_HOST 0
#define MPG_MEM_DEVICE 1

/* pinocchio joint models (pinocchio 2.6.21 JointCollectionDefault subset) */
#define MPG_JOINT_RX 0
#define MPG_JOINT_RY 1
#define MPG_JOINT_RZ 2
#define MPG_JOINT_REVOLUTE_UNALIGNED 3
#define MPG_JOINT_PX 4
#define MPG_JOINT_PY 5
#define MPG_JOINT_PZ 6
#define MPG_JOINT_PRISMATIC_UNALIGNED 7
#define MPG_JOINT_RUBX 8  /* continuous joints: user value v -> (cos v, sin v) */
#define MPG_JOINT_RUBY 9
#define MPG_JOINT_RUBZ 10
#define MPG_JOINT_RUB_UNALIGNED 11

/* FCL geometry kinds supported on the device */
#define MPG_GEOM_CONVEX 0   /* fcl::Convex   : vertices, param = first face
                               int, face count (convex_face)             */
#define MPG_GEOM_BOX 1      /* fcl::Box      : param = side x, y, z          */
#define MPG_GEOM_SPHERE 2   /* fcl::Sphere   : param = radius                */
#define MPG_GEOM_CAPSULE 3  /* fcl::Capsule  : param = radius, lz            */
#define MPG_GEOM_CYLINDER 4 /* fcl::Cylinder : param = radius, lz            */
#define MPG_GEOM_OCTREE 5   /* fcl::OcTree   : param = first leaf, leaf count,
                               resolution; static, on a link or attached;
                               a pair of two OcTrees collides (leaf OBBs),
                               its contacts / distance are refused      */
#define MPG_GEOM_MESH 6     /* fcl::BVHModel<OBBRSS> (non-convex mesh):
                               vertices, param = first triangle, triangle
                               count (mesh_triangle)                     */
#define MPG_GEOM_ELLIPSOID 7 /* fcl::Ellipsoid : param = radii a, b, c
                                (python/pybind_fcl.hpp:137-141); libccd
                                supportEllipsoid, MPR with every partner */
#define MPG_GEOM_CONE 8      /* fcl::Cone : param = radius, lz, apex at
                                +lz/2 (python/pybind_fcl.hpp:95-98); libccd
                                supportCone, MPR with every partner       */
#define MPG_GEOM_TRIANGLE 9  /* fcl::TriangleP : vertices a, b, c (vertex
                                count 3, python/pybind_fcl.hpp:168-175);
                                libccd supportTriangle / centerTriangle,
                                MPR with every shape (not paired with an
                                OcTree or BVH mesh)                        */

/*
 * World descriptor.  SE3 values are 12 doubles: a row-major 3x3 rotation
 * followed by the translation.  All arrays are read during
 * mpg_world_create only.
 */
typedef struct mpg_world_desc {
  /* --- kinematics: pinocchio joints 1..n_joints (universe omitted) ------- */
  int32_t n_joints;
  const int32_t *joint_type;     /* MPG_JOINT_*                               */
  const int32_t *joint_parent;   /* parent joint, 0 = universe, else 1-based  */
  const double *joint_axis;      /* [n_joints*3] (unaligned joints only)      */
  const double *joint_placement; /* [n_joints*12] model.jointPlacements       */
  /* joint value source: dof slot d >= 0 reads q[i*dof + d]; -1 uses
   * joint_value_const (fixed, non-move-group joints keep current_qpos_,
   * src/articulated_model.cpp:104-113).                                    */
  const int32_t *joint_q_source; /* [n_joints]                             */
  const double *joint_q_const;   /* [n_joints]                             */
  int32_t dof;                   /* move-group dimension = row length of q */

  /* --- user links (PinocchioModel::setLinkOrder) ---------------------------- */
  int32_t n_links;
  const int32_t *link_parent;     /* frame.parent joint (0 = universe)      */
  const double *link_placement;   /* [n_links*12] frame.placement           */

  /* --- geometry ------------------------------------------------------------- */
  int32_t n_geoms;
  const int32_t *geom_type;       /* MPG_GEOM_*                             */
  const int32_t *geom_vertex_start;
  const int32_t *geom_vertex_count;
  const double *geom_param;       /* [n_geoms*4]                            */
  int64_t n_vertices;
  const double *vertices;         /* [n_vertices*3] Convex vertices, local  */

  /* --- moving objects: robot collision objects then attached bodies -------- */
  int32_t n_moving;
  const int32_t *moving_link;     /* user link index                        */
  const int32_t *moving_geom;
  const double *moving_offset;    /* [n_moving*12] link -> object pose      */

  /* --- static scene objects -------------------------------------------------- */
  int32_t n_static;
  const int32_t *static_geom;
  const double *static_transform; /* [n_static*12] world pose               */

  /* --- pairs, in output-bit order. Object ids: [0, n_moving) moving,
   *     [n_moving, n_moving + n_static) static.  (pair_a[p], pair_b[p]) keeps
   *     fcl::collide's (o1, o2) argument order.                              */
  int32_t n_pairs;
  const int32_t *pair_a;
  const int32_t *pair_b;
  const uint8_t *pair_allowed;    /* 1: ACM allows it (never reported)      */

  /* --- CollisionRequest -------------------------------------------------------- */
  double gjk_tolerance;           /* CollisionRequest::gjk_tolerance (1e-6) */

  /* --- octrees (MPG_GEOM_OCTREE): the occupied leaves of every octree
   *     geometry as axis-aligned boxes in the octree frame, [min xyz, max xyz]
   *     per leaf, as fcl::OcTree's getRootBV / computeChildBV recursion
   *     yields them (PlanningWorldTpl::addPointCloud, planning_world.cpp:102-110) */
  int64_t n_octree_leaves;
  const double *octree_leaf;      /* [n_octree_leaves*6]                    */

  /* --- BVH meshes (MPG_GEOM_MESH, load_mesh_as_BVH, src/urdf_utils.cpp:
   *     136-155): triangles as three vertex indices relative to the mesh's
   *     geom_vertex_start */
  int64_t n_mesh_triangles;
  const int32_t *mesh_triangle;   /* [n_mesh_triangles*3]                   */

  /* --- convex faces: fcl::Convex(vertices, num_faces, faces) keeps them and
   *     FCL 0.7.0 derives its support from them (Convex::findExtremeVertex
   *     walks the face graph when the hull has more than 32 vertices and the
   *     faces are watertight: src/urdf_utils.cpp:156-183 builds every link hull
   *     that way).  FCL layout: count, count vertex indices (relative to the
   *     geometry's geom_vertex_start), count, ...  For MPG_GEOM_CONVEX,
   *     geom_param[0] = first int of the geometry's faces in convex_face,
   *     geom_param[1] = number of faces (0 = no faces: linear support).     */
  int64_t n_convex_face_ints;
  const int32_t *convex_face;     /* [n_convex_face_ints]                   */

  /* --- joint limits (PinocchioModelTpl::getJointLimit, src/pinocchio_model.cpp:
   *     59-83): [lower, upper] of each joint value, -inf / +inf or NULL =
   *     unbounded.  Only the broad phase reads them: the travel of a prismatic
   *     move-group joint bounds the fp32 cull's coordinates.  A configuration
   *     outside them is still evaluated exactly (every pair of it goes to the
   *     narrow phase), so no input changes a result.                         */
  const double *joint_lower;      /* [n_joints] or NULL                     */
  const double *joint_upper;      /* [n_joints] or NULL                     */

  /* --- CollisionRequest::gjk_solver_type (python/pybind_fcl.hpp:264, 276):
   *     MPG_GJK_LIBCCD (0, the default, libccd MPR in float) or MPG_GJK_INDEP
   *     (FCL's own GJK in double, GJKSolver_indep::shapeIntersect) for every
   *     shape pair without an FCL closed form.  GST_INDEP worlds take shape
   *     geometry only (MPG_GEOM_OCTREE / MPG_GEOM_MESH in a non-allowed pair:
   *     MPG_E_UNSUPPORTED) and the collide entry points only (contacts:
   *     MPG_E_UNSUPPORTED; the distance calls keep libccd, as
   *     DistanceRequest's own default does).                               */
  int32_t gjk_solver;
} mpg_world_desc;

#define MPG_GJK_LIBCCD 0
#define MPG_GJK_INDEP 1

typedef struct mpg_world mpg_world;

typedef struct mpg_world_info {
  int32_t n_pairs;
  int32_t mask_words; /* uint32 words per configuration in pair_mask      */
  int32_t dof;
  int32_t n_links;
  int32_t device;
  int32_t block_size;
  int64_t snapshot_bytes;
} mpg_world_info;

/* Build an immutable device snapshot of the world on `device`. */
int mpg_world_create(const mpg_world_desc *desc, int device, mpg_world **out);
int mpg_world_destroy(mpg_world *world);
int mpg_world_get_info(const mpg_world *world, mpg_world_info *info);

/*
 * q:         [n*dof] row-major move-group joint values (float64).
 * flags:     [n] 1 if the configuration collides (collide() == true).
 * pair_mask: [n*mask_words] bit p of word p/32 set if pair p is reported by
 *            collideFull(); may be NULL when only flags are wanted.
 */
int mpg_collide_batch(mpg_world *world, const double *q, int64_t n, uint8_t *flags,
                      uint32_t *pair_mask, int mem, void *stream);

/*
 * One host batch over several GPUs: worlds[k] (each from mpg_world_create of
 * the same descriptor, on its own device) checks the k-th contiguous shard of
 * q (the first n % n_worlds shards one row longer), all shards concurrently
 * from host threads, results written in place -- isValid is a pure function
 * of the state (src/ompl_planner.h:59-62), so no collective is involved.
 * Host buffers only; the first failing world's status is returned.  The
 * in-process counterpart of mplib_amd.dist (one process per GPU).
 */
int mpg_collide_batch_multi(mpg_world *const *worlds, int32_t n_worlds, const double *q, int64_t n,
                            uint8_t *flags, uint32_t *pair_mask);

/*
 * The shard of a batch of n configurations that part k of n_parts checks:
 * contiguous, the first n % n_parts shards one row longer (the split of
 * mpg_collide_batch_multi and of mplib_amd.dist.shard_range).  Host only.
 */
int mpg_shard_range(int64_t n, int32_t k, int32_t n_parts, int64_t *start, int64_t *count);

/*
 * Device-resident multi-GPU batch: shard k is already on worlds[k]'s device
 * -- q[k] [counts[k] * dof], flags[k] [counts[k]], pair_mask[k]
 * [counts[k] * mask_words] (pair_mask or pair_mask[k] NULL: flags only) --
 * and is enqueued on streams[k] (a hipStream_t of that device; streams or
 * streams[k] NULL: its default stream), one host thread per world; no host
 * round trip, no synchronisation (as MPG_MEM_DEVICE calls).
 * gather_flags / gather_masks (device pointers on worlds[0]'s device, NULL:
 * no gather): every shard's flags / mask rows are also copied there, shard k
 * at row counts[0] + ... + counts[k-1], device to device (peer copies over
 * xGMI on streams[k]); streams[0] then waits for all of them, so work queued
 * on streams[0] after the call sees the whole batch.  The worlds must come
 * from the same descriptor (checked by the snapshot's hash) and be distinct.
 * isValid is a pure function of the state (src/ompl_planner.h:59-62): no
 * collective is involved in the check itself.
 */
int mpg_collide_batch_multi_device(mpg_world *const *worlds, int32_t n_worlds, const double *const *q,
                                   const int64_t *counts, uint8_t *const *flags, uint32_t *const *pair_mask,
                                   void *const *streams, uint8_t *gather_flags, uint32_t *gather_masks);

/*
 * Host-buffer calls (mem == MPG_MEM_HOST) of at most `n` configurations take
 * the latency path: one launch with one wave per (pair, 64-configuration tile)
 * and one synchronisation, instead of the throughput pipeline (6 launches).
 * Identical results; default 1024 (env MPG_SMALL_BATCH_MAX), 0 disables.
 * The planner's validity batches (mplib_amd OMPLPlanner) are this size.
 */
int mpg_set_small_batch_max(mpg_world *world, int64_t n);

/*
 * Drops the device state the world keeps for one caller stream (its phase
 * A/B workspace and the internal side stream of large batches).  Call before
 * destroying a stream that was passed to MPG_MEM_DEVICE calls; without it the
 * state of at most 32 streams is kept, least recently used evicted first.
 * No reference counterpart (the reference has no device state).
 */
int mpg_release_stream(mpg_world *world, void *stream);

/*
 * Same pair evaluation as mpg_collide_batch, but the link poses are given
 * directly instead of being computed from joint values:
 * link_pose [n*n_links*7] = (px, py, pz, qw, qx, qy, qz) per user link.
 * Replaces FCLModelTpl::updateCollisionObjects(vector<Vector7>)
 * (src/fcl_model.cpp:151-167) followed by FCLModelTpl::collideFull
 * (src/fcl_model.cpp:182-193).
 */
int mpg_collide_link_poses(mpg_world *world, const double *link_pose, int64_t n, uint8_t *flags,
                           uint32_t *pair_mask, int mem, void *stream);

/*
 * Batched motion validation: for each edge e, OMPL's
 * DiscreteMotionValidator::checkMotion(q_from[e], q_to[e]) over MPlib's state
 * space (src/ompl_planner.cpp:248-293: one RealVectorStateSpace(1) per
 * prismatic/revolute joint, SO2StateSpace for continuous joints, weights 1):
 *   segments[e] = max(1, ceil(distance / longest_valid_segment)),
 *   states q(j/segments), j = 1..segments (the last is q_to itself; q_from is
 *   assumed valid, as OMPL does), each checked with collide().
 *   valid[e] = 1 if every state is collision-free;
 *   first_invalid[e] = smallest colliding j, or -1 (checkMotion's lastValid).
 * so2_mask: bit i set if move-group dof i is an SO2 subspace.  first_invalid
 * and segments may be NULL.  Synchronises `stream` once (the state count
 * sizes the work).
 */
int mpg_check_motion_batch(mpg_world *world, const double *q_from, const double *q_to, int64_t n,
                           uint32_t so2_mask, double longest_valid_segment, uint8_t *valid,
                           int32_t *first_invalid, int32_t *segments, int mem, void *stream);

/*
 * Batched distance: per configuration, PlanningWorldTpl::distanceSelf and
 * distanceOthers (src/planning_world.cpp:493-720) over the pair table, whose
 * first n_self_pairs entries form the self group: ACM-allowed pairs are
 * skipped, each pair's fcl::distance(o1 = pair_a, o2 = pair_b, request) is
 * compared with strict '<' (:513), so the first minimum wins.
 * d_*: minimum distance (DBL_MAX if the group is empty), p_*: its pair
 * index (-1 if none).  What fcl::distance computes [FCL 0.7.0, restated in
 * oracle/collide_oracle.c pair_distance and oracle/fcl_gjk_dist.h]:
 *   shape-shape   DistanceRequest(): GJKSolver_libccd::shapeDistance -- the
 *                 closed forms for sphere-sphere / -box / -capsule /
 *                 -cylinder (either order) and capsule-capsule, else
 *                 GJKDistance: libccd's GJK (__ccdGJK, then _ccdDist) in float
 *                 (ccd_real_t of the reference's libccd build), -1 once GJK
 *                 finds the shapes intersecting.  With enable_signed_distance
 *                 every shape pair runs GJKSignedDistance: GJK, then for
 *                 intersecting shapes FCL's EPA (__ccdEPA to epa_tolerance
 *                 1e-4, penEPAPosClosest): -(penetration depth).  One
 *                 departure: where FCL's EPA would expand a nearest face the
 *                 new support point does not see (its polytope turns
 *                 non-convex and can cycle forever), the EPA stops at that
 *                 face (oracle/fcl_gjk_dist.h, "convexity guard").
 *   OcTree-shape  the minimum over the occupied leaves of shapeDistance(Box
 *                 (leaf), shape) (OcTreeShapeDistanceRecurse).
 *   mesh-shape    the minimum over the triangles of shapeTriangleDistance
 *                 (sphereTriangleDistance for spheres, else GJK on the
 *                 triangle GJK object) (MeshShapeDistanceTraversalNodeOBBRSS).
 *   mesh-mesh     the minimum of triDistance over the triangle pairs (0 when
 *                 one intersects) (MeshDistanceTraversalNodeOBBRSS).
 *   mesh-OcTree   the minimum over (leaf box, triangle) of GJK distance
 *                 (OcTreeMeshDistanceRecurse).
 *   Mesh and OcTree pairs are unsigned whatever the request (their leaves
 *   call the unsigned shapeDistance / triDistance), -1 once a leaf test
 *   penetrates.
 * Device and oracle agree bit for bit on the GJK/EPA floats; between equal
 * minima of a mesh / OcTree pair the first leaf test in the oracle's scan
 * order wins (FCL's RSS-ordered traversal may pick another equal one).
 */
int mpg_distance_batch(mpg_world *world, const double *q, int64_t n, int32_t n_self_pairs, double *d_self,
                       int32_t *p_self, double *d_others, int32_t *p_others, int mem, void *stream);

/*
 * DistanceRequest (python/pybind_fcl.hpp:310-316) as PlanningWorldTpl::
 * distance* passes it to fcl::distance (src/planning_world.cpp:512, 537):
 *   flags: MPG_DISTANCE_SIGNED (enable_signed_distance),
 *          MPG_DISTANCE_NEAREST_POINTS (enable_nearest_points),
 *          MPG_DISTANCE_GJK_INDEP (gjk_solver_type = GST_INDEP);
 *   distance_tolerance: GJKSolver_libccd::distance_tolerance, libccd's
 *          dist_tolerance (default 1e-6).
 * pts_self / pts_others ([n*6], may be NULL): DistanceResult::nearest_points
 * [0] and [1] (world frame) of each group's minimum pair, as FCL leaves them:
 *   shape-shape   always (the shape leaf computes them whatever the flags):
 *                 points on o1 and o2; zeros for an unsigned penetration (-1);
 *   OcTree-shape  always, (leaf box point, shape point) in that order for
 *                 both argument orders (the tree is the traversal's o1);
 *   mesh-shape    always; (mesh point, shape point), swapped to (shape, mesh)
 *                 for a (shape, mesh) pair only with enable_nearest_points;
 *   mesh-mesh     only with enable_nearest_points (zeros otherwise);
 *   mesh-OcTree   always, (leaf box point, triangle point).
 * Where FCL throws (its EPA's FCL_THROW_FAILED_AT_THIS_CONFIGURATION) the
 * configuration's p_self = p_others = MPG_DISTANCE_FCL_THROWS and both
 * distances are NaN; MPG_MEM_HOST calls then return MPG_E_FAILED.  An EPA
 * that outgrows the lane's private polytope (96 vertices) is run again from
 * the start with a 2048-vertex polytope from a per-world pool; only past
 * that is the configuration marked MPG_DISTANCE_EPA_CAPACITY (MPG_MEM_HOST:
 * MPG_E_UNSUPPORTED) -- never a silently different value.
 */
#define MPG_DISTANCE_SIGNED 1
#define MPG_DISTANCE_NEAREST_POINTS 2
#define MPG_DISTANCE_GJK_INDEP 4 /* gjk_solver_type = GST_INDEP: FCL's own GJK
                                    in double (ShapeDistanceIndepImpl, its
                                    gjk_tolerance = distance_tolerance) for
                                    the shape pairs without a closed form;
                                    unsigned only, no OcTree / BVH mesh pair
                                    (MPG_E_UNSUPPORTED)                   */
#define MPG_DISTANCE_FCL_THROWS (-2)
#define MPG_DISTANCE_EPA_CAPACITY (-3)
typedef struct mpg_distance_request {
  int32_t flags;
  double distance_tolerance;
} mpg_distance_request;
int mpg_distance_batch_req(mpg_world *world, const double *q, int64_t n, int32_t n_self_pairs,
                           const mpg_distance_request *request, double *d_self, int32_t *p_self, double *pts_self,
                           double *d_others, int32_t *p_others, double *pts_others, int mem, void *stream);
/* mpg_distance_batch_req with distance_tolerance = 1e-6 */
int mpg_distance_batch_ex(mpg_world *world, const double *q, int64_t n, int32_t n_self_pairs, int32_t flags,
                          double *d_self, int32_t *p_self, double *pts_self, double *d_others, int32_t *p_others,
                          double *pts_others, int mem, void *stream);

/*
 * Collide with contacts: CollisionRequest(enable_contact=True).  Same flags /
 * pair_mask as mpg_collide_batch (input_kind MPG_INPUT_Q: q rows) or
 * mpg_collide_link_poses (MPG_INPUT_LINK_POSES), plus, for every reported
 * pair p of configuration i, libccd's MPR penetration (FCL GJKCollide ->
 * ccdMPRPenetration, the one contact FCL reports for an MPR pair):
 *   depth[i*P + p], normal[(i*P + p)*3 ..] (from object 1 to object 2),
 *   pos[(i*P + p)*3 ..]; zeros for pairs not reported.  P = n_pairs.
 * FCL closed-form pairs report the contact FCL 0.7's specialisation emits
 * (box-box: boxBox2's clipped face points / edge-edge closest point, with its
 * stored penetration_depth = -(point depth) <= 0; sphere-sphere; sphere-box
 * and box-sphere; sphere-capsule; sphere-cylinder; the shape-sphere orders
 * flip the normal), reduced to the one contact ShapeShapeCollide keeps for
 * num_max_contacts = 1.  A point-cloud (OcTree) pair reports the contact of
 * the first occupied leaf of FCL's traversal that intersects the shape, with
 * the tree as the contact's o1 (normal from the leaf box into the shape).
 * A BVH-mesh pair reports the contact of the first intersecting leaf test
 * in FCL 0.7.0's traversal order of its BVHModel<OBBRSS> tree (the tree is
 * rebuilt as FCL builds it, and only leaf tests FCL's OBB tests let through
 * count): mesh-shape the smallest leaf position (left child first), with the
 * sphere-triangle contact or libccd MPR penetration of (shape, triangle);
 * mesh-mesh the pair whose descent (first tree descended when the second
 * node is a leaf or the first is larger) is lexicographically first, with
 * intersect_Triangle's deepest point of the shallower triangle (o1's frame ->
 * world); mesh-OcTree the first in OcTreeMeshIntersectRecurse's interleaved
 * descent (octree children 0..7, mesh left then right), MPR penetration of
 * (leaf box, triangle).
 */
#define MPG_INPUT_Q 0
#define MPG_INPUT_LINK_POSES 1
int mpg_collide_contacts(mpg_world *world, const double *input, int64_t n, int input_kind, uint8_t *flags,
                         uint32_t *pair_mask, double *depth, double *normal, double *pos, int mem, void *stream);

/* link_pose: [n*n_links*7] = getLinkPose(l) -> (px, py, pz, qw, qx, qy, qz). */
int mpg_fk_batch(mpg_world *world, const double *q, int64_t n, double *link_pose, int mem,
                 void *stream);

/*
 * Per-kernel timing with HIP events recorded on the launch stream (off by
 * default; no cost when off).  mpg_profile_read synchronises the recorded
 * events, writes the accumulated milliseconds, launch counts and work units
 * of each stage since the last read (then resets them).  Units: configurations
 * for CULL and BUCKET, narrow-phase (configuration, pair) candidates for
 * NARROW.  Any output pointer may be NULL.
 *   MPG_STAGE_CULL    phase A broad phase           (cull_kernel)
 *   MPG_STAGE_BUCKET  survivor bucketing            (tile_count/pair_scan/chunk_scan/scatter)
 *   MPG_STAGE_NARROW  phase B exact narrow phase    (narrow_kernel)
 */
#define MPG_STAGE_CULL 0
#define MPG_STAGE_BUCKET 1
#define MPG_STAGE_NARROW 2
#define MPG_NUM_STAGES 3
int mpg_profile_enable(mpg_world *world, int enable);
int mpg_profile_read(mpg_world *world, double *ms, int64_t *launches, int64_t *units, int n_stages);

/*
 * Diagnostics: fcl::collide(geometry geom_a at Ta[i], geometry geom_b at
 * Tb[i]) for i < n (SE3 as 12 doubles each; host buffers), through the same
 * narrow-phase dispatch as mpg_collide_batch (FCL closed form, octree / BVH
 * mesh walk, or libccd MPR) -- the narrow phase without forward kinematics,
 * for parity tests against the CPU restatement.  hit[i] = 1 on contact.
 */
int mpg_debug_collide_pairs(mpg_world *world, int32_t geom_a, int32_t geom_b, int64_t n, const double *Ta,
                            const double *Tb, uint8_t *hit);

/*
 * Planner.generate_collision_pair (mplib/planner.py:118-163), batched: n
 * configurations of the world's state drawn uniformly in [lower, upper]
 * (dof values each) on the device, evaluated as mpg_collide_batch does, and
 * counts[p] (host, n_pairs) = how many of them report pair p (collide_full()
 * of the sample).  The reference loops set_qpos(random, full=True) +
 * collide_full() 10^6 times on the host; build the world with every joint of
 * the planned articulations as a state value for that semantics.
 * Sampler: value i of the batch (row-major) is lower + (upper - lower) * u,
 * u = (splitmix64(seed + (i + 1) * 0x9E3779B97F4A7C15) >> 11) * 2^-53;
 * mpg_sample_uniform returns the same values (host buffer, rows counted from
 * row_offset).  dof <= 64.
 */
int mpg_collide_count(mpg_world *world, const double *lower, const double *upper, int64_t n, uint64_t seed,
                      int64_t *counts, void *stream);
int mpg_sample_uniform(const double *lower, const double *upper, int32_t dof, int64_t n, uint64_t seed,
                       int64_t row_offset, double *q, int device);

/*
 * Diagnostics (host only, no device): the FCL 0.7.0 BVHModel<OBBRSS> tree the
 * snapshot builds for a BVH mesh (BVHModel::endModel -> buildTree:
 * BVFitter<OBBRSS>::fit, SPLIT_METHOD_MEAN; OBB half), whose OBB tests gate
 * mesh pairs as FCL's traversal does.  boxes [(2T - 1) * 15] = per node the
 * row-major axis matrix (columns = box axes), centre, half extents; links
 * [(2T - 1) * 3] = first child node (-(triangle + 1) for a leaf), first leaf
 * position, leaf count; leaf_order [T] = primitive_indices after the build.
 * Returns the node count (2T - 1) or a negative status.
 */
int mpg_fcl_bvh_build(const double *vertices, int32_t n_vertices, const int32_t *triangles, int32_t n_triangles,
                      double *boxes, int32_t *links, int32_t *leaf_order);

/* Diagnostics: the device sin/cos used by the FK (host buffers). */
int mpg_debug_sincos(const double *x, int64_t n, double *s, double *c, int device);

/*
 * Latency server accounting (the resident kernel behind host batches of at
 * most MPG_SMALL_SERVER_MAX states): batches it answered,
 * times it was (re)started, calls that fell back to one launch per batch
 * because it could not be started or did not answer.  state: 0 = not used by
 * this world (MPG_SMALL_SERVER=0, or pairs it does not serve), 1 = in use,
 * 2 = fallen back (it is tried again one second after the failure).  Any
 * output pointer may be NULL.  No reference counterpart (diagnostics).
 */
int mpg_latency_server_stats(mpg_world *world, int64_t *served, int64_t *starts, int64_t *fallbacks,
                             int32_t *state);

/* Synchronise the world's device (used after MPG_MEM_DEVICE calls). */
int mpg_synchronize(int device);

int mpg_device_count(int *count);
const char *mpg_last_error(void);
/*
 * The last error text of the calling thread copied into buf (at most size - 1
 * bytes and a terminating NUL; truncated if longer).  Returns the full length
 * of the text (excluding the NUL), as snprintf does, so a caller can size a
 * buffer; buf may be NULL when size is 0.  This is SURVEY.md 8(b)'s
 * mpg_last_error(char*, size_t) form for bindings that cannot hold a pointer
 * into library-owned thread-local storage (cgo / JNI); mpg_last_error() above
 * stays for C and ctypes callers.
 */
int mpg_last_error_copy(char *buf, size_t size);
const char *mpg_version(void);

#ifdef __cplusplus
}
#endif
#endif /* MPGPU_H */
