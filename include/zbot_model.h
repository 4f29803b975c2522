/*
 * zbot_model.h — compiled robot descriptor ("ZbModel") shared by the HIP engine
 * (libzbot_hip.so) and the CPU oracle (oracle/liboracle_zbot.so).
 *
 * This is a *data format*, the equivalent of the subset of MuJoCo's mjModel that
 * the Z-Bot walking task touches (reference: train.py:1326-1331 loads the Z-Bot
 * MJCF through MuJoCo C; MuJoCo 3.3.4 `mjModel` field names are reused below so a
 * maintainer can map them 1:1). It is filled on the host by the Python
 * descriptor compiler (ksim-gym-zbot_amd/zbot_amd/model.py) from a JSON robot
 * description and copied verbatim to device memory, where one workgroup stages
 * it into LDS.
 *
 * Restrictions (checked by the compiler, see model.py::compile_model):
 *   - a kinematic tree with at most one joint per body; joint types: free
 *     (root only) or hinge; other bodies are welded (no joint);
 *   - nbody <= ZB_MAX_BODY, nv <= ZB_MAX_DOF, dof-chain depth <= ZB_MAX_DEPTH;
 *   - collision = floor plane (world geom) vs up to ZB_MAX_GEOM = 16 per-body boxes,
 *     capsules, cylinders, spheres, ellipsoids or convex meshes (<= ZB_MAX_MESHV hull
 *     vertices each; the two foot soles first by
 *     convention); of the robot's own pairs only the two box soles against each
 *     other (npair <= 1, box-box, alone or beside other floor colliders); any
 *     other self pair is counted in nskip_pair and refused;
 *   - actuators = motors on hinge joints (joint transmission, gear).
 * All floats are fp32; all vectors are padded to 4 so rows are 16-B aligned.
 */
#ifndef ZBOT_MODEL_H
#define ZBOT_MODEL_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZB_MODEL_MAGIC   0x5A424F54u /* 'ZBOT' */
#define ZB_MODEL_VERSION 9

#define ZB_MAX_BODY  32
#define ZB_MAX_DOF   32
#define ZB_MAX_QPOS  40
#define ZB_MAX_DEPTH 12
#define ZB_MAX_GEOM  16  /* floor colliders (model v9; the engine collides the two soles and, per substep,
                            the first four others within reach of the floor, two beside the sole pair:
                            DESIGN.md §4j) */
#define ZB_MAX_MESHV 64  /* convex hull vertices of one mesh collider */
#define ZB_MAX_MESHVERT 512 /* the mesh vertex pool (all mesh colliders together) */
#define ZB_MAX_SITE  8
#define ZB_MAX_ACT   32
#define ZB_CON_PER_GEOM 4 /* plane-box at most 4 corners, plane-cylinder 4, plane-mesh 4, plane-capsule 2, plane-sphere / -ellipsoid 1 */
#define ZB_CON_PER_PAIR 4 /* box-box (the sole pair): at most 4 contacts */
#define ZB_MAX_CON  (ZB_MAX_GEOM * ZB_CON_PER_GEOM)

/* joint types (mjtJoint values where they exist) */
#define ZB_JNT_NONE  -1
#define ZB_JNT_FREE   0
#define ZB_JNT_HINGE  3

/* collider types (mjtGeom values) */
#define ZB_GEOM_SPHERE  2
#define ZB_GEOM_CAPSULE 3
#define ZB_GEOM_ELLIPSOID 4
#define ZB_GEOM_CYLINDER 5
#define ZB_GEOM_BOX     6
#define ZB_GEOM_MESH    7 /* a convex mesh: the hull's vertices (geom_vertadr / geom_vertnum / mesh_vert) */

typedef struct ZbModel {
  /* header */
  uint32_t magic;
  int32_t  version;
  int32_t  struct_bytes;
  int32_t  nbody, nq, nv, nu, ngeom, nsite;
  int32_t  max_depth;            /* max over dofs of dof_depth + 1 */

  /* options (mjOption subset) */
  float    gravity[4];           /* opt.gravity */
  float    timestep;             /* opt.timestep (train.py:1777 dt=0.001) */
  float    meaninertia;          /* mjStatistic.meaninertia (solver scale) */
  float    pad_opt[2];

  /* bodies (index 0 = world) */
  int32_t  body_parent[ZB_MAX_BODY];
  int32_t  body_depth[ZB_MAX_BODY];     /* world 0, root 1, ... */
  int32_t  body_jnttype[ZB_MAX_BODY];   /* ZB_JNT_* */
  int32_t  body_dofadr[ZB_MAX_BODY];    /* first dof of this body's joint or -1 */
  int32_t  body_dofnum[ZB_MAX_BODY];
  int32_t  body_qposadr[ZB_MAX_BODY];
  int32_t  body_lastdof[ZB_MAX_BODY];   /* deepest dof of the chain from root to here (-1: none) */
  float    body_pos[ZB_MAX_BODY][4];    /* frame offset in parent frame */
  float    body_quat[ZB_MAX_BODY][4];   /* frame rotation rel. parent (w,x,y,z) */
  float    body_ipos[ZB_MAX_BODY][4];   /* com in body frame */
  float    body_iquat[ZB_MAX_BODY][4];  /* principal inertia frame */
  float    body_mass[ZB_MAX_BODY][4];   /* [0]=mass, [1]=subtree mass */
  float    body_inertia[ZB_MAX_BODY][4];/* principal inertia diag */
  float    body_invweight0[ZB_MAX_BODY][4]; /* [0]=translational, [1]=rotational */

  /* joints (at most one per body; indexed by body) */
  float    jnt_axis[ZB_MAX_BODY][4];    /* hinge axis, body frame */
  float    jnt_pos[ZB_MAX_BODY][4];     /* anchor, body frame */

  /* dofs */
  int32_t  dof_body[ZB_MAX_DOF];
  int32_t  dof_parent[ZB_MAX_DOF];      /* mjModel.dof_parentid */
  int32_t  dof_depth[ZB_MAX_DOF];       /* position in the root->dof chain */
  int32_t  dof_anc[ZB_MAX_DOF][ZB_MAX_DEPTH]; /* ancestor dof at each depth (self at own depth), -1 beyond */
  int32_t  dof_limited[ZB_MAX_DOF];
  int32_t  dof_qposadr[ZB_MAX_DOF];     /* hinge: qpos index, free: -1 */
  float    dof_armature[ZB_MAX_DOF];
  float    dof_damping[ZB_MAX_DOF];
  float    dof_frictionloss[ZB_MAX_DOF];
  float    dof_invweight0[ZB_MAX_DOF];
  float    dof_range[ZB_MAX_DOF][2];
  float    dof_solref[4];               /* shared by frictionloss + limit rows */
  float    dof_solimp[8];               /* dmin dmax width mid power */

  float    qpos0[ZB_MAX_QPOS];          /* mjModel.qpos0 (hinges: joint zero) */
  float    pad_q[4];

  /* actuators: motor, joint transmission. ctrl index order == qpos[7:] order
     (train.py:1358-1359 orders the Feetech parameter vectors by ctrl index and
      train.py:1252-1253 compares them with qpos[7:]) */
  int32_t  act_dof[ZB_MAX_ACT];
  float    act_gear[ZB_MAX_ACT];
  float    act_ctrlrange[ZB_MAX_ACT][2];
  /* Feetech servo parameters per actuator (train.py:1121-1134, 1396-1414) */
  float    fe_kp[ZB_MAX_ACT];
  float    fe_kd[ZB_MAX_ACT];
  float    fe_error_gain[ZB_MAX_ACT];
  float    fe_max_pwm[ZB_MAX_ACT];
  float    fe_vin[ZB_MAX_ACT];
  float    fe_kt[ZB_MAX_ACT];
  float    fe_R[ZB_MAX_ACT];
  float    fe_vmax[ZB_MAX_ACT];
  float    fe_amax[ZB_MAX_ACT];
  float    fe_max_torque[ZB_MAX_ACT];    /* stored, never applied (train.py:1221) */
  float    fe_max_velocity[ZB_MAX_ACT];

  /* collision geoms colliding with the floor plane z=0 */
  int32_t  geom_body[ZB_MAX_GEOM];
  int32_t  geom_type[ZB_MAX_GEOM];      /* ZB_GEOM_* */
  float    geom_pos[ZB_MAX_GEOM][4];
  float    geom_quat[ZB_MAX_GEOM][4];
  float    geom_size[ZB_MAX_GEOM][4];    /* mjModel.geom_size: box half sizes; capsule / cylinder
                                           radius, half-length (local z); sphere radius; mesh: the
                                           largest vertex distance from the geom origin (a bound) */
  /* floor: geom_priority=2 (train.py:1330) -> floor friction/solref/solimp win */
  float    floor_friction[4];            /* sliding, torsional, rolling */
  float    floor_solref[4];
  float    floor_solimp[8];
  float    floor_margin;
  float    pad_floor[3];

  /* the robot's own colliding pair the engine simulates (npair 0 or 1): the two box soles against
     each other (box-box). The contact normal points from geom pair_geom[0] to pair_geom[1] (MuJoCo's
     geom1 -> geom2). Parameters as MuJoCo mixes them for two geoms of equal priority
     (mj_contactParam): friction the larger of the two per component, solref / solimp the mean
     (solmix 1 each), margin the larger. */
  int32_t  npair;
  int32_t  pair_geom[2];
  float    pair_margin;
  float    pair_friction[4];
  float    pair_solref[4];
  float    pair_solimp[8];

  /* sites */
  int32_t  site_body[ZB_MAX_SITE];
  float    site_pos[ZB_MAX_SITE][4];
  float    site_quat[ZB_MAX_SITE][4];

  /* named entities the task uses (train.py:1453,1495-1520,662-663) */
  int32_t  site_imu;        /* "imu_site" */
  int32_t  site_left_foot;  /* "left_foot"  */
  int32_t  site_right_foot; /* "right_foot" */
  int32_t  body_base;       /* floating base, body 1 */
  int32_t  body_left_foot;  /* "Left_Foot"  */
  int32_t  body_right_foot; /* "Right_Foot" */
  int32_t  geom_left_foot;  /* touch sensor zone of left_foot site */
  int32_t  geom_right_foot;

  /* derived topology tables (filled by the descriptor compiler, read by the
     HIP engine so no per-launch scans are needed) */
  int32_t  max_body_depth;
  int32_t  mrow_size;                  /* packed depth-indexed row storage (floats) */
  int32_t  nskip_geom;                 /* colliding geoms of the source model the engine cannot
                                          collide (other types, or past ZB_MAX_GEOM): zb_create
                                          rejects nskip_geom > 0 */
  int32_t  nskip_pair;                 /* robot geom pairs the source model collides with each
                                          other (contype / conaffinity, MuJoCo's filters): the
                                          engine has floor contacts only, so zb_create rejects
                                          nskip_pair > 0 */
  int32_t  body_nchild[ZB_MAX_BODY];
  int32_t  body_child[ZB_MAX_BODY][8]; /* -1 padded */
  int32_t  depth_maxchild[16];         /* max #children over bodies at a depth */
  uint32_t dof_desc[ZB_MAX_DOF];       /* bitmask of strict descendant dofs */
  uint32_t dof_ancpk[ZB_MAX_DOF][4];   /* dof_anc as bytes: byte (e&3) of word e>>2 */
  uint32_t dof_rowmask[ZB_MAX_DOF];    /* contact rows (16 per geom, geoms 0-1) whose chain holds the dof */
  int32_t  dof_act[ZB_MAX_DOF];        /* actuator driving the dof or -1 */
  int32_t  dof_rowoff[ZB_MAX_DOF];     /* offset of the dof's row in packed storage */
  int32_t  geom_lastdof[ZB_MAX_GEOM];
  /* elimination levels of the sparse L'DL (level = height of the dof in the
     dof tree; dofs of one level are never ancestor/descendant of each other,
     so they are eliminated together) */
  int32_t  nlevel;
  int32_t  pad_lvl[3];
  int32_t  level_nmem[ZB_MAX_DEPTH];
  int32_t  level_mem[ZB_MAX_DEPTH][8];

  /* task constants: JOINT_BIASES (train.py:61-82), ctrl order */
  float    joint_bias[ZB_MAX_ACT];
  float    joint_weight[ZB_MAX_ACT];

  /* convex mesh colliders (ZB_GEOM_MESH, model v8): geom g's hull vertices are
     mesh_vert[geom_vertadr[g] .. + geom_vertnum[g]] in the geom frame, in the order MJX's plane_convex
     scans them (its manifold selection breaks ties by index) */
  int32_t  geom_vertadr[ZB_MAX_GEOM];
  int32_t  geom_vertnum[ZB_MAX_GEOM];
  float    mesh_vert[ZB_MAX_MESHVERT][4];
  float    pad_end[4];
} ZbModel;

#ifdef __cplusplus
}
#endif
#endif /* ZBOT_MODEL_H */
