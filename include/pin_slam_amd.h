/*
 * pin_slam_amd.h -- C ABI of the MI355X (gfx950) neural-point SDF engine.
 *
 * The reference (kelly7707/PIN_SLAM) has no FFI: its hot path is the Python
 * class API of model.neural_points.NeuralPoints / model.decoder.Decoder
 * evaluated by PyTorch ATen ops.  Each entry point below replaces one piece of
 * that path (reference file:line cited per function); the Python package
 * pin_slam_amd binds them with ctypes and restores the reference's class API.
 *
 * Conventions
 *   - every pointer is a DEVICE pointer unless its comment says host;
 *   - the library keeps no state and caches no pointer between calls;
 *   - every call is stream-ordered on `stream` (a hipStream_t passed as void*),
 *     never synchronises, and returns PIN_OK or a negative PIN_ERR_* code;
 *   - sizes are int64_t element counts.
 */
#ifndef PIN_SLAM_AMD_H
#define PIN_SLAM_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PIN_OK 0
#define PIN_ERR_ARG (-1)         /* bad argument (null pointer, size, unsupported shape) */
#define PIN_ERR_HIP (-2)         /* a HIP launch or runtime call failed */
#define PIN_ERR_UNSUPPORTED (-3) /* configuration outside what the kernels implement */

#define PIN_FEATURE_DIM 8        /* feature_dim of every reference config */
#define PIN_MAX_NN_K 8           /* query_nn_k <= 8 in every reference config */
#define PIN_HIDDEN_DIM 64        /* geo_mlp_hidden_dim, geo_mlp_level = 1 */
#define PIN_RECORD_UNFAITHFUL (1 << 30) /* record id flag, see pin_build_records */

/* Voxel hash + neighbourhood (model/neural_points.py:69-73, :430-457, :459-476). */
typedef struct PinHash {
    const int32_t* table;        /* [buffer_size] slot -> global point index, -1 empty */
    int64_t buffer_size;         /* B, < 2^31 */
    float resolution;            /* voxel size; points are floor(p / resolution) in f32 */
    int32_t num_cells;           /* Kc */
    const int32_t* cells;        /* [pin_cells_padded(Kc)]: floor_mod(dx*p0+dy*p1+dz*p2, B) per cell, 0-padded */
    float max_valid_dist2;       /* candidates with dist2 > this are rejected (f32 compare) */
    int32_t reserved;
} PinHash;

/* Per-point candidate records and the arrays the k nearest neighbours are read from. */
typedef struct PinPoints {
    const float* records;        /* [M,4]: x, y, z, bits(id); id -1 = rejected (see pin_build_records) */
    int64_t num_points;          /* M */
    const float* features;       /* [rows, 8] geo features addressed by id */
    const float* positions;      /* [rows, 3] positions addressed by id (read for flagged records) */
    const float* orientations;   /* [rows, 4] quaternions (w,x,y,z); read only if after_pgo */
    const float* certainties;    /* [rows] */
    int64_t rows;
    int32_t after_pgo;           /* rotate neighbour vectors (model/neural_points.py:606-607) */
    int32_t reserved;
    const float* positions4;     /* [rows, 4] x, y, z, pad: the same positions as 16-B rows, or NULL.  Set:
                                    pin_train_forward reads each neighbour's position with one 16-B
                                    load beside its feature loads (all by id) instead of three 4-B ones */
} PinPoints;

/* Occupancy-grid box: origin cell (ox,oy,oz) and extent in 4x4x4-cell bricks. */
typedef struct PinGridDims {
    int64_t ox, oy, oz;
    int32_t nbx, nby, nbz;
    int32_t reserved;
} PinGridDims;

/* Occupancy grid + compact per-cell arrays in brick order (see pin_grid_mark / pin_grid_fill). */
typedef struct PinGrid {
    const uint32_t* bricks;      /* [nb,4]: bits lo, bits hi, exclusive prefix, 0 */
    PinGridDims dims;
    const float* crec;           /* [n_occ,4]: x, y, z, bits(id) of the cell's point (its record) */
    const int32_t* cgid;         /* [n_occ] global point index of each compact record */
    int64_t n_occ;
    const int32_t* offsets;      /* [pin_cells_padded(Kc)] packed (dx+128) | (dy+128)<<8 | (dz+128)<<16,
                                    then num_columns column entries (see num_columns) */
    float resolution;
    int32_t num_cells;           /* Kc, reference cell order (model/neural_points.py:430-439) */
    float max_valid_dist2;
    const float* cfeat;          /* [n_occ,8] features in brick order (fat), else NULL */
    const float* ccert;          /* [n_occ] certainties in brick order (fat), else NULL */
    int32_t fat;                 /* 1: features/certainty read from cfeat/ccert; 0: from PinPoints by id */
    int32_t window;              /* max |offset| component (num_nei_cells); <= 2 enables the
                                    brick-window scan (<= 8 bricks cover the neighbourhood) */
    int32_t num_columns;         /* 0, or the cells regrouped as (x, y) columns: entry c at
                                    offsets[pin_cells_padded(Kc) + c] = (dx+128) | (dy+128)<<8 |
                                    (dz0+128)<<16 | nz<<24 covers cells dz0 .. dz0+nz-1 of the
                                    column; the columns in order list exactly the cells in order */
} PinGrid;

/* Geo decoder, hidden_level = 1 (model/decoder.py:16-88). */
typedef struct PinMlp {
    const float* W1;             /* [64, 11] */
    const float* b1;             /* [64] */
    const float* W2;             /* [1, 64] */
    const float* b2;             /* [1] */
    float sdf_scale;             /* logistic_gaussian_ratio * sigma_sigmoid_m (decoder.py:51-54) */
    int32_t reserved;
    const void* packed;          /* PIN_MLP_PACK_BYTES written by pin_mlp_pack from THESE weights, or NULL.
                                    Set: the SDF kernels (pin_query_sdf*) decode on the f16 matrix cores
                                    when the gradient is requested (each f32 operand split into two f16
                                    terms, f32 accumulation), as do pin_train_forward under PIN_TRAIN_DX
                                    and pin_train_backward's per-neighbour path without mlp_grad;
                                    NULL (or SDF only): f32 VALU */
} PinMlp;

/*
 * pin_mlp_pack -- the decoder as MFMA operand tiles (pin_query_sdf_grid*, decoder.py:66-88):
 *   GEMM1  P^T = [W1 | b1] [x ; 1]       64 hidden x 64 queries of a wave, K = 11 + bias
 *   GEMM2  g^T = (W1 o w2)^T 1[P > 0]    rows 0..10: dsdf/dx_i / s, row 11: sum_c 1[P_c>0] w2_c b1_c,
 *                                        so that sdf = s (x . g + row 11 + b2)  (= s (w2 . relu(P) + b2))
 * Each f32 operand v is stored as v_hi + v_lo (f16, round to nearest) after a power-of-two
 * scale per operand row (rows of W1|b1 and of W1 o w2 to [2^13, 2^14); queries scaled per
 * lane in the kernel): products are exact in the f32 accumulators and the dropped lo*lo term
 * is ~2^-22 relative, the f32 rounding level of the reference's own sums.  Inputs |x| < 2^29.
 * Re-run after every decoder update (Mapper steps change W1/b1/W2/b2).
 */
#define PIN_MLP_PACK_BYTES 8288
int pin_mlp_pack(const PinMlp* mlp, void* packed, void* stream);

/*
 * pin_build_records -- per-point candidate records for one query mode.
 * Replaces the per-candidate work of model/neural_points.py:480-499 + :555:
 *   record[g] = (x_g, y_g, z_g, id_g) with
 *     query_locally == 0:  id_g = g
 *     query_locally == 1:  id_g = -1 if |travel_dist[cur_ts] - travel_dist[ts_create[g]]|
 *                                      >= diff_travel_dist_local   (time filter, :480-488)
 *                          id_g = global2local[g] otherwise          (:555)
 *   and, if id_g >= 0 and local_positions[id_g] != positions[g] bitwise, id_g |= PIN_RECORD_UNFAITHFUL
 *   (the neighbour vector then reads the local position; the distance keeps the global one).
 */
int pin_build_records(const float* positions, int64_t num_points, int32_t query_locally,
                      const int64_t* global2local, const int64_t* ts_create, const float* travel_dist,
                      int64_t travel_len, int64_t cur_ts, float diff_travel_dist_local,
                      const float* local_positions, int64_t local_rows, float* records, void* stream);

/* Cell-delta table length for Kc cells: Kc rounded up to a multiple of 16. */
static inline int32_t pin_cells_padded(int32_t num_cells) { return (num_cells + 15) / 16 * 16; }

/* pin_neighbor_cells -- fill the cell-delta table (pin_cells_padded(Kc) int32) from host
 * offsets [Kc,3] (neural_points.py:430-439): slot(cell + dx) = floor_mod(base + delta, B). */
int pin_neighbor_cells(const int32_t* host_dx, int32_t num_cells, int64_t buffer_size,
                       int32_t* cells_out, void* stream);

/*
 * pin_hash_rebuild -- table[slot(p_i)] = i for i in [0,n), the highest i winning a shared slot
 * (model/neural_points.py:420-422, recreate_hash with merged points).  The table must be
 * filled with -1 by the caller.
 */
int pin_hash_rebuild(const float* positions, int64_t n, float resolution, int32_t* table,
                     int64_t buffer_size, void* stream);

/*
 * pin_radius_search -- model/neural_points.py:459-509 for the records' mode:
 * dist2 [n,Kc] f32 (max_valid_dist2 for rejected) and idx [n,Kc] int64 (global index or -1).
 */
int pin_radius_search(const PinHash* hash, const PinPoints* pts, const float* q, int64_t n,
                      float* dist2_out, int64_t* idx_out, void* stream);

/*
 * pin_query_sdf -- fused query_feature + Decoder.sdf + analytic dSDF/dq for inference
 * (utils/tracker.py:176-260 query_source_points, utils/mesher.py:41-136 query_points,
 * utils/tools.py:174 get_gradient).  Outputs may be NULL when not wanted:
 *   sdf [n], grad [n,3], nn_count [n] int32, certainty [n], sdf_std [n] (weighted_first == 0).
 * zero_empty != 0 gives rows without neighbours sdf 0 (mesher) instead of MLP(0).
 */
int pin_query_sdf(const PinHash* hash, const PinPoints* pts, const PinMlp* mlp, const float* q, int64_t n,
                  int32_t nn_k, int32_t weighted_first, int32_t zero_empty, float* sdf, float* grad,
                  int32_t* nn_count, float* certainty, float* sdf_std, void* stream);

/*
 * pin_query_feature_fwd -- model/neural_points.py:528-674 forward (inference outputs):
 *   feat [n,11] (weighted_first) or [n,nn_k,11]; weights [n,nn_k]; nn_counts [n] int64;
 *   certainty [n]; saved local ids [n,nn_k] int32 and global ids [n,nn_k] int32 (-1 invalid).
 */
int pin_query_feature_fwd(const PinHash* hash, const PinPoints* pts, const float* q, int64_t n, int32_t nn_k,
                          int32_t weighted_first, float* feat, float* weights, int64_t* nn_counts,
                          float* certainty, int32_t* ids, int32_t* gids, void* stream);

/*
 * pin_query_feature_bwd -- backward of pin_query_feature_fwd given dL/dfeat and dL/dweights
 * (either may be NULL): grad_q [n,3] (may be NULL) and grad_features [rows,8] accumulated
 * with float atomics (may be NULL).  The reference obtains these from autograd through
 * model/neural_points.py:492-662.
 */
int pin_query_feature_bwd(const PinPoints* pts, const float* q, int64_t n, int32_t nn_k, int32_t weighted_first,
                          const int32_t* ids, const int32_t* gids, const float* weights, const float* grad_feat,
                          const float* grad_weights, float* grad_q, float* grad_features, void* stream);

/*
 * pin_query_feature_bwd2 -- the double backward of pin_query_feature_bwd (second-order autograd:
 * get_gradient(..., create_graph=True), utils/tools.py:174-184, through model/neural_points.py:
 * 577-662): given the first backward's inputs (ids, gids, weights, grad_feat G, grad_weights Gw;
 * G / Gw may be NULL) and the upstream gradients of its outputs, up_q = dL2/dgrad_q [n,3] and
 * up_features = dL2/dgrad_features [rows,8] (either may be NULL), it writes dL2/dq [n,3],
 * dL2/dG (grad_feat's shape), dL2/dGw [n,nn_k] (each may be NULL) and, weighted_first only, adds
 * dL2/dfeatures into d_features [rows,8] with float atomics (may be NULL).  Closed form per query
 * (pin_query.hip, k_query_feature_bwd2).
 */
int pin_query_feature_bwd2(const PinPoints* pts, const float* q, int64_t n, int32_t nn_k, int32_t weighted_first,
                           const int32_t* ids, const int32_t* gids, const float* weights, const float* grad_feat,
                           const float* grad_weights, const float* up_q, const float* up_features, float* d_q,
                           float* d_grad_feat, float* d_grad_weights, float* d_features, void* stream);

/*
 * pin_train_scatter -- training-mode side effects of query_feature (model/neural_points.py:637-648):
 * certainties[id] += w (scatter_add_), ts_update[id] = max(ts_update[id], query_ts) (scatter_reduce amax,
 * only if query_ts and ts_update are non-NULL).
 */
int pin_train_scatter(const int32_t* ids, const float* weights, int64_t n, int32_t nn_k, const int64_t* query_ts,
                      float* certainties, int64_t* ts_update, void* stream);

/*
 * pin_query_certainty -- model/neural_points.py:511-525: max certainty over the cells of the
 * hash's neighbourhood (own voxel in utils/mapper.py:283), 0 where empty.
 */
int pin_query_certainty(const PinHash* hash, const PinPoints* pts, const float* q, int64_t n,
                        float* certainty_out, void* stream);

/* Registration validity / robust-weight parameters (utils/tracker.py:277-394). */
typedef struct PinRegParams {
    int32_t min_nn_count;        /* mask = nn_count >= query_nn_k (:286-287) */
    float min_grad_norm;         /* reg_min_grad_norm */
    float max_grad_norm;         /* reg_max_grad_norm */
    float max_sdf_std;           /* surface_sample_range_m * max_sdf_std_ratio (only if sdf_std given) */
    float gm_dist;               /* reg_GM_dist_m, <= 0: no residual weight */
    float gm_grad;               /* reg_GM_grad, <= 0: no gradient weight */
    int32_t div_grad_norm;       /* reg_dist_div_grad_norm: r = sdf / |g| - label (:335-336) */
    int32_t q4_points;           /* 1: points are pin_query_sort rows {x, y, z, bits(i)} with sdf / grad /
                                    nn_count / sdf_std in the same (tile) order (PIN_QUERY_OUT_TILE);
                                    sdf_label and valid_out stay indexed by the original i */
} PinRegParams;

/* accumulator layout of pin_reg_normal_eq's output */
#define PIN_REG_NACC 31          /* [0] sum w, [1] sum |r|, [2] sum w r^2, [3] n_valid,
                                    [4..24] sum w J^T J (upper triangle, row major),
                                    [25..30] sum w r J,  J = [p x g, g] */
#define PIN_REG_WORKSPACE_DOUBLES (256 * PIN_REG_NACC + 8)   /* block partials, then pin_reg_step's counter
                                                             (one word that must be ZERO before the first
                                                             pin_reg_step on a workspace; it is left zero) */

/*
 * pin_reg_normal_eq -- fused validity mask + Geman-McClure weights + f64 normal-equation
 * accumulation of one registration step (utils/tracker.py:303-394 and implicit_reg :468-480),
 * deterministic (fixed-order two-level reduction).  sdf_std / sdf_label may be NULL (no std
 * test / zero labels); valid_out (n bytes, may be NULL) receives the validity mask.
 * weight != NULL: every point is valid and w_i = weight[i] (implicit_reg on pre-filtered,
 * pre-weighted rows, :468-496); nn_count may then be NULL.
 * out[PIN_REG_NACC] doubles (device); workspace PIN_REG_WORKSPACE_DOUBLES doubles.
 */
int pin_reg_normal_eq(const float* points, const float* sdf, const float* grad, const int32_t* nn_count,
                      const float* sdf_std, const float* sdf_label, const float* weight, int64_t n,
                      const PinRegParams* prm, double* workspace, double* out, uint8_t* valid_out, void* stream);

/* Status record of pin_reg_solve (doubles). */
#define PIN_REG_NSTATUS 8        /* [0] n_valid, [1] mean |r| in cm, [2] rotation of dT in degrees,
                                    [3] |translation of dT| m, [4] 1 if solved (n_valid >= 10) */

/*
 * pin_reg_solve -- implicit_reg's 6x6 solve on the device (utils/tracker.py:483-496, expmap
 * :580-589) from pin_reg_normal_eq's accumulators: N += lm_lambda diag(N), t = N^-1 g in f64,
 * delta_pose [4,4] f64 = [expmap(t[0:3]) | t[3:6]] (identity below 10 valid points, :310-312);
 * pose_out = delta_pose @ pose_in when both are non-NULL (the tracking loop's T = dT T, :115);
 * status[PIN_REG_NSTATUS] as above (the rotation angle is :132's, rotation_matrix_to_axis_angle).
 */
int pin_reg_solve(const double* acc, double lm_lambda, const double* pose_in, double* delta_pose, double* pose_out,
                  double* status, void* stream);

/*
 * pin_reg_step -- pin_reg_normal_eq (sdf_label / sdf_std may be NULL; no weights, no valid_out)
 * followed by pin_reg_solve in ONE launch: the last block to finish sums the block partials in
 * pin_reg_normal_eq's fixed order (bitwise the same acc) and solves.  acc [PIN_REG_NACC], status,
 * delta_pose, pose_in / pose_out as pin_reg_solve; workspace PIN_REG_WORKSPACE_DOUBLES doubles whose
 * counter word is zero before the first call.
 */
int pin_reg_step(const float* points, const float* sdf, const float* grad, const int32_t* nn_count,
                 const float* sdf_std, const float* sdf_label, int64_t n, const PinRegParams* prm, double* workspace,
                 double* acc, double lm_lambda, const double* pose_in, double* delta_pose, double* pose_out,
                 double* status, void* stream);

/* pin_transform_points -- transform_torch (utils/tools.py:386-399): out [n,3] f32 = the points
 * under pose [4,4] (row-major f64 on the device, cast to f32), one fma chain per coordinate. */
int pin_transform_points(const float* points, int64_t n, const double* pose, float* out, void* stream);

/* pin_transform_points_sorted -- the same transform into pin_query_sort rows, in place: row k of
 * q4 [n,4] becomes {pose * points[i], bits(i)} with i = bits(q4[4k+3]) kept.  The tracking loop
 * sorts its source cloud once per call and re-poses the sorted rows on later iterations (the tile
 * order is a locality hint; results do not depend on it). */
int pin_transform_points_sorted(const float* points, int64_t n, const double* pose, float* q4, void* stream);

/*
 * pin_reg_iteration -- one iteration of Tracker.tracking (utils/tracker.py:92-159) in one call,
 * stream-ordered, no host synchronisation:
 *   1. the source cloud under pose_in: first iteration with q4 != NULL (grid only) -> posed into
 *      cur and tile-sorted into q4 (order_ws as pin_query_sort); later ones -> q4 re-posed in place
 *      (pin_transform_points_sorted); q4 == NULL -> posed into cur;
 *   2. the fused SDF + dSDF/dq query (grid or hash; outputs in tile order when sorted);
 *   3.+4. pin_reg_step (prm.q4_points is set from the sorted flag): the accumulators into
 *      acc_status_dt[0..30], status into [31..38], dT into [39..54], pose_out = dT pose_in;
 *   5. host_out != NULL (pinned host, 55 doubles): an asynchronous copy of the 55 doubles.
 * Exactly one of grid / hash is non-NULL.  pose_in / pose_out: [4,4] f64 device, distinct.
 */
typedef struct PinRegIter {
    const float* src;            /* [n,3] source points (f32) */
    int64_t n;
    const float* labels;         /* [n] sdf labels by source index, or NULL (zeros) */
    float* cur;                  /* [n,3] scratch: the posed cloud */
    float* q4;                   /* [n,4] tile-sorted rows (grid, sorted mode) or NULL */
    void* order_ws;              /* pin_query_order_workspace_bytes(n), zeroed state (first sorted iteration) */
    float* sdf;                  /* [n] */
    float* grad;                 /* [n,3] */
    int32_t* nn_count;           /* [n] */
    float* sdf_std;              /* [n], read when weighted_first == 0 */
    double* reg_ws;              /* PIN_REG_WORKSPACE_DOUBLES, counter word zeroed (pin_reg_step) */
    double* acc_status_dt;       /* device: PIN_REG_NACC + PIN_REG_NSTATUS + 16 doubles */
    double* host_out;            /* pinned host copy target (55 doubles) or NULL */
    int32_t nn_k;
    int32_t weighted_first;
    double lm_lambda;
    PinRegParams prm;
} PinRegIter;
int pin_reg_iteration(const PinGrid* grid, const PinHash* hash, const PinPoints* pts, const PinMlp* mlp,
                      const PinRegIter* it, int32_t first, const double* pose_in, double* pose_out, void* stream);

/*
 * pin_cell_bounds -- out[0..2] = min, out[3..5] = max over the points of floor(p / resolution)
 * (f32 division, the reference's voxel rule, neural_points.py:214); the occupancy-grid box.
 * Empty input leaves out = {INT64_MAX x3, INT64_MIN x3}.
 */
int pin_cell_bounds(const float* positions, int64_t num_points, float resolution, int64_t* out, void* stream);

/* Workspace bytes pin_grid_mark needs for a grid of nb bricks. */
static inline int64_t pin_grid_workspace_bytes(int64_t num_bricks) {
    return ((num_bricks + 4095) / 4096) * 4 + 16;
}

/*
 * pin_grid_mark -- build the occupancy bricks of the map box: bit(cell) = 1 iff some point g
 * has floor(p_g / res) == cell and table[slot(cell)] == g ("own-cell" entries), then the
 * per-brick exclusive prefix of the bit counts.  counters[0] = own-cell entries marked,
 * counters[1] = occupied table slots.  The grid equals the table on every candidate that
 * can pass the distance test iff counters[0] == counters[1] (no displaced entries, e.g.
 * after adjust_map without recreate_hash) and no two cells within the reachable window
 * collide under the hash (host check).  workspace: pin_grid_workspace_bytes(nb) bytes.
 */
int pin_grid_mark(const float* positions, int64_t num_points, float resolution, const int32_t* table,
                  int64_t buffer_size, const PinGridDims* dims, uint32_t* bricks, unsigned long long* counters,
                  void* workspace, void* stream);

/* pin_grid_mark with flags: PIN_GRID_TABLE_TRUSTED -- the caller vouches that every occupied table
 * slot holds a point at its own cell's slot (the table was written from the current positions by
 * pin_map_insert / pin_hash_assign / pin_hash_rebuild and nothing moved since), so counters[1] =
 * counters[0] without the pass over the B-slot table. */
#define PIN_GRID_TABLE_TRUSTED 1
int pin_grid_mark_ex(const float* positions, int64_t num_points, float resolution, const int32_t* table,
                     int64_t buffer_size, const PinGridDims* dims, uint32_t* bricks, unsigned long long* counters,
                     void* workspace, int32_t flags, void* stream);

/*
 * pin_grid_fill -- compact arrays in brick order for one query mode, for every own-cell point g
 * at rank r = rank(cell_g): crec[r] = record_g, cgid[r] = g and, when cfeat / ccert are
 * non-NULL, cfeat[r] = features[id_g], ccert[r] = certainty[id_g] (zeros for rejected records).
 */
int pin_grid_fill(const float* positions, int64_t num_points, float resolution, const int32_t* table,
                  int64_t buffer_size, const PinGridDims* dims, const uint32_t* bricks, const float* records,
                  const float* features, const float* certainties, float* crec, float* cfeat, float* ccert,
                  int32_t* cgid, void* stream);

/* Workspace of pin_query_order / pin_query_sort: PIN_ORDER_STATE_BYTES of state (per-tile
 * totals and a done counter) that must be ZERO before the first call on a workspace and that
 * every call leaves zero again (calls sharing one workspace must be ordered on one stream), then
 * 8 bytes per query. */
#define PIN_ORDER_STATE_BYTES 65600   /* up to 16384 tiles: 4 B per tile + the counter line */
static inline int64_t pin_query_order_workspace_bytes(int64_t n) {
    return PIN_ORDER_STATE_BYTES + 8 * n;
}

/*
 * pin_query_order -- a processing order for a random query batch: order[0..n) is a permutation
 * of the query indices grouped into <= 4096 spatial tiles of the grid box (a counting sort:
 * two launches, one returning global atomic per (block, tile)).  Feeding it to
 * pin_query_sdf_grid gives better line sharing and per-XCD L2 locality; results do not depend
 * on the order (the order inside a tile is not deterministic).
 */
int pin_query_order(const PinGrid* grid, const float* q, int64_t n, int32_t* order, void* workspace, void* stream);

/*
 * pin_query_sort -- the same tile sort, writing the queries themselves in tile order:
 * q4[4 * pos .. 4 * pos + 3] = {x, y, z, bits(i)} (int32 index i in the last float's bits);
 * order (may be NULL) as pin_query_order.  Input of pin_query_sdf_grid_sorted.
 */
int pin_query_sort(const PinGrid* grid, const float* q, int64_t n, float* q4, int32_t* order, void* workspace,
                   void* stream);

/*
 * pin_query_sort_stable -- pin_query_sort's tiles (same tile map), but a STABLE sort: inside a
 * tile the queries keep their input order, so the processing order is a function of the batch
 * alone (the deterministic training mode: per-block decoder-gradient partials and per-wave loss
 * partials then sum the same rows in the same order on every run).  A radix sort of the tile keys
 * (rocPRIM, several launches): slower than the counting sort.  workspace:
 * pin_query_sort_stable_workspace_bytes(n) bytes, no state kept between calls.
 */
int64_t pin_query_sort_stable_workspace_bytes(int64_t n);
int pin_query_sort_stable(const PinGrid* grid, const float* q, int64_t n, float* q4, int32_t* order, void* workspace,
                          void* stream);

/*
 * pin_query_sdf_grid -- pin_query_sdf with candidates from the occupancy grid.  order (n ints,
 * may be NULL = input order): the order in which queries are processed (pin_query_order);
 * outputs always go to each query's own index.
 */
int pin_query_sdf_grid(const PinGrid* grid, const PinPoints* pts, const PinMlp* mlp, const float* q, int64_t n,
                       int32_t nn_k, int32_t weighted_first, int32_t zero_empty, float* sdf, float* grad,
                       int32_t* nn_count, float* certainty, float* sdf_std, const int32_t* order, void* stream);

/*
 * pin_query_sdf_grid_sorted -- pin_query_sdf_grid over queries pre-sorted by pin_query_sort
 * (q4 [n,4]: coordinates + original index); outputs go to each query's original index.
 */
int pin_query_sdf_grid_sorted(const PinGrid* grid, const PinPoints* pts, const PinMlp* mlp, const float* q4,
                              int64_t n, int32_t nn_k, int32_t weighted_first, int32_t zero_empty, float* sdf,
                              float* grad, int32_t* nn_count, float* certainty, float* sdf_std, void* stream);

/*
 * pin_query_sdf_grid_tiled -- pin_query_sort into q4 ([n,4] f32 scratch) followed by
 * pin_query_sdf_grid_sorted, in one call (the launches leave the host back to back);
 * workspace as pin_query_order.  Outputs go to each query's own index.
 */
int pin_query_sdf_grid_tiled(const PinGrid* grid, const PinPoints* pts, const PinMlp* mlp, const float* q,
                             int64_t n, int32_t nn_k, int32_t weighted_first, int32_t zero_empty, float* sdf,
                             float* grad, int32_t* nn_count, float* certainty, float* sdf_std, float* q4,
                             void* workspace, void* stream);

/* flags of the _ex forms: outputs in tile order -- element k of sdf / grad / nn_count / certainty /
 * sdf_std belongs to the query q4[k] (original index bits(q4[4k+3])) -- instead of at each query's
 * own index: coalesced stores, for consumers that reduce over the queries (the tracker's normal
 * equations, pin_reg_normal_eq with PinRegParams.q4_points) or read the index from q4 */
#define PIN_QUERY_OUT_TILE 1

/* pin_query_sdf_grid_tiled / pin_query_sdf_grid_sorted with flags (PIN_QUERY_OUT_TILE); every
 * argument is checked before the sort is launched. */
int pin_query_sdf_grid_tiled_ex(const PinGrid* grid, const PinPoints* pts, const PinMlp* mlp, const float* q,
                                int64_t n, int32_t nn_k, int32_t weighted_first, int32_t zero_empty, float* sdf,
                                float* grad, int32_t* nn_count, float* certainty, float* sdf_std, float* q4,
                                void* workspace, int32_t flags, void* stream);
int pin_query_sdf_grid_sorted_ex(const PinGrid* grid, const PinPoints* pts, const PinMlp* mlp, const float* q4,
                                 int64_t n, int32_t nn_k, int32_t weighted_first, int32_t zero_empty, float* sdf,
                                 float* grad, int32_t* nn_count, float* certainty, float* sdf_std, int32_t flags,
                                 void* stream);

/* pin_query_feature_fwd_grid -- pin_query_feature_fwd with candidates from the occupancy grid
 * (features always read live from pts->features; gids from grid->cgid). */
int pin_query_feature_fwd_grid(const PinGrid* grid, const PinPoints* pts, const float* q, int64_t n, int32_t nn_k,
                               int32_t weighted_first, float* feat, float* weights, int64_t* nn_counts,
                               float* certainty, int32_t* ids, int32_t* gids, void* stream);

/* One mapping iteration (utils/mapper.py:443-572): the main batch of n_main rows and the
 * numerical-gradient stencil of 6*n_stencil rows generated from coord[::decimation]
 * (mapper.py:683-711; row n_main + b*n_stencil + k is coord[k*decimation] +- eps along axis
 * b/2, + for even b). */
typedef struct PinTrainCfg {
    int64_t n_main;              /* N, rows of the batch */
    int64_t n_stencil;           /* ceil(N / decimation), 0 disables the eikonal term */
    int32_t decimation;          /* gradient_decimation */
    int32_t nn_k;                /* query_nn_k */
    int32_t weighted_first;
    float eps;                   /* float32(voxel_size_m * num_grad_step_ratio) */
    float sigma;                 /* BCE scale, Mapper.sdf_scale (mapper.py:521, loss.py:40-47) */
    float weight_e;              /* eikonal weight (mapper.py:547) */
    float grad_scale;            /* multiplies loss and gradients: 1, or 1/world_size so that a SUM
                                    all-reduce of per-rank gradients is the gradient of the mean loss */
    int32_t flags;               /* PIN_TRAIN_ROWS: `coord` of pin_train_forward holds every row (batch and
                                    stencil, pin_train_rows / pin_train_gather) instead of the batch;
                                    PIN_TRAIN_DX (mlp->packed set, no decoder gradient): weighted_first --
                                    the forward decodes on the matrix cores and saves s dsdf/dx[0:8] as
                                    x [rows, 8] instead of the input, and the backward applies it without
                                    re-evaluating the decoder; per-neighbour -- the forward saves each
                                    neighbour's 64 ReLU masks as x [rows, nn_k] uint64 instead of its
                                    vector, and the backward's input gradients are the matrix-core
                                    decoder's second GEMM over them (no feature re-gather, no hidden
                                    layer);
                                    PIN_TRAIN_EIK: analytic-gradient eikonal (numerical_grad off,
                                    mapper.py:481-482, get_gradient create_graph=True, tools.py:174-184):
                                    n_stencil must be 0; the forward evaluates dsdf/dq of every batch row in
                                    closed form, its loss weight_e * mean(|g| - 1)^2 and the coefficients of
                                    its second derivative (st->eik_coef / eik_vec), and the backward adds
                                    them to the feature / decoder gradients */
    int64_t n_tail;              /* the last n_tail batch rows (and the stencil groups based on them) are
                                    scaled by grad_scale_tail instead of grad_scale (slab sharding) */
    float grad_scale_tail;
    int32_t reserved;
} PinTrainCfg;

#define PIN_TRAIN_ROWS 1
#define PIN_TRAIN_DX 2
#define PIN_TRAIN_EIK 4
/* PIN_TRAIN_PAIR: pin_train_forward runs two lanes per row where it can (grid backend with the
 * column scan, weighted_first, a packed decoder): the row's candidate list split between the two,
 * the halves merged in reference order -- the same neighbours, ids, weights, sdf and saved state
 * as one lane per row, with twice the waves for a batch of ~1 wave per SIMD (small batches). */
#define PIN_TRAIN_PAIR 8

/* Per-row buffers saved by pin_train_forward for pin_train_backward (rows = n_main + 6 n_stencil). */
typedef struct PinTrainState {
    int32_t* ids;                /* [rows, nn_k] local feature rows, -1 invalid */
    float* weights;              /* [rows, nn_k] IDW weights */
    float* x;                    /* weighted_first: [rows, 11] decoder input (PIN_TRAIN_DX: [rows, 8] s dsdf/dx
                                    over the features); else [rows, nn_k, 3] vectors (PIN_TRAIN_DX:
                                    the buffer read as [rows, nn_k] uint64 ReLU masks) */
    float* sdf;                  /* [rows] predicted sdf */
    float* certainties;          /* [L] += w (training side effect, neural_points.py:640), may be NULL;
                                    applied by pin_train_backward from ids / weights */
    int64_t* ts_update;          /* [L] amax with the batch rows' ts (row_ts, neural_points.py:644), may be
                                    NULL; applied by pin_train_backward */
    const int32_t* order;        /* [rows] processing order (pin_query_order over pin_train_rows), may be
                                    NULL; ids/weights/x are stored per processing slot, sdf per row */
    const float* sorted_rows;    /* [rows,4] the rows in processing order as {x, y, z, bits(row)}
                                    (pin_query_sort over the rows), may be NULL; takes precedence over
                                    order and saves the order -> coordinate dependent load */
    const float* row_weight;     /* [n_main] BCE weight per batch row (loss_weight_on: |weight|,
                                    mapper.py:514-516, loss.py:41-42), NULL = unweighted */
    float* eik_coef;             /* PIN_TRAIN_EIK: [rows, nn_k] per slot, u . dw_j/dq with
                                    u = dL_eik/dg (the neighbour weights' share of the second derivative) */
    float* eik_vec;              /* PIN_TRAIN_EIK: weighted_first: [rows, 11] A^T u = sum_j (u . dw_j/dq) x_j
                                    + (sum_j w_j) [0, u] (decoder-parameter term, written only when
                                    the decoder trains); per-neighbour: [rows, 3] u */
    const int64_t* row_ts;       /* [n_main] the batch rows' ts (the `ts` of pin_train_forward), read by
                                    pin_train_backward for the ts_update side effect; NULL: none */
    float* grad_replicas;        /* optional, with replicas > 1: [replicas, L+1, 8] f32 scratch, zero on the
                                    first call; pin_train_backward scatters block b's feature terms into
                                    replica b % replicas, then adds the replicas into grad_features and
                                    zeroes them again.  For small batches on small maps, whose most
                                    referenced points serialise the memory-side float atomics on one
                                    address line; NULL / replicas <= 1: straight into grad_features */
    int32_t replicas;
    int32_t replica_mode;        /* 0: pin_train_backward adds the replicas into grad_features itself;
                                    1: it leaves them, and the caller's pin_adam_step_train takes the
                                    gradient as grad_features + the replicas' sum (one launch less) */
    /* Deterministic accumulation: with grad_fixed non-NULL the feature
     * terms are added as 64-bit fixed-point integers into grad_fixed [2, max(replicas, 1), L+1, 8]
     * (zero on the first call) instead of float atomics into grad_features / grad_replicas: a term
     * with |term| 2^fixed_shift >= 4096 as round(term 2^fixed_shift) into the first (coarse) part, a
     * smaller one as round(term 2^(fixed_shift + 40)) into the second (fine) part, so gradients down
     * to ~1e-27 keep their value (the reference's Adam, eps 1e-15, steps on gradients of 1e-18).  Integer addition is associative, so the sum does not depend on
     * the order the atomics arrive in: the gradient is a function of the batch alone, bitwise.  It
     * reaches grad_features as float(coarse 2^-fixed_shift + fine 2^-(fixed_shift + 40)) through
     * pin_train_backward (replica_mode
     * 0) or pin_adam_step_train (replica_mode 1), which zero the integers again.  With cert_fixed
     * non-NULL the certainty side effect goes the same way into cert_fixed [L] (shift cert_shift),
     * and the caller folds it into the certainties with pin_fixed_accumulate (certainties is then
     * not written).  Terms beyond +-2^(62 - shift) saturate. */
    int64_t* grad_fixed;
    int64_t* cert_fixed;
    int32_t fixed_shift;         /* e.g. 50: resolution 8.9e-16, range +-8192 */
    int32_t cert_shift;          /* e.g. 32 */
} PinTrainState;

/* Scalars of one torch.optim.Adam step (utils/tools.py:111-112; betas (0.9, 0.99)). */
typedef struct PinAdamStep {
    float neg_step_size;         /* float32(-lr / (1 - beta1^t)) */
    float one_minus_beta1;       /* lerp weight */
    float beta2;
    float one_minus_beta2;
    float bias_correction2_sqrt; /* float32(sqrt(1 - beta2^t)) */
    float eps;                   /* adam_eps */
    int32_t zero_grad;           /* bit 0: grad := 0 after the step (opt.zero_grad of the next iteration);
                                    bit 1: the first step of a fresh optimiser -- exp_avg / exp_avg_sq
                                    are taken as zero, not read (they may hold anything) */
    int32_t grad_stride;         /* element i's gradient is grad[(i/8)*grad_stride + i%8] (8: contiguous) */
} PinAdamStep;

/* decoder-parameter gradient layout of pin_train_backward's mlp_grad */
#define PIN_MLP_GRAD_SIZE (PIN_HIDDEN_DIM * (PIN_FEATURE_DIM + 3) + 2 * PIN_HIDDEN_DIM + 1) /* W1,b1,W2,b2 */

/*
 * The drop-in Decoder.sdf (model/decoder.py:66-88, the 11 -> 64 -> 1 ReLU decoder with bias)
 * on rows and its autograd, for callers that go through NeuralPoints.query_feature + Decoder.sdf
 * (utils/mapper.py:448-573 with autograd, utils/tools.py:174-184 get_gradient):
 *
 * pin_mlp_forward -- out[r] = s (w2 . relu(W1 x_r + b1) + b2), x [n, 11], s = mlp->sdf_scale.
 *
 * pin_mlp_backward -- with m_c(r) = [W1[c] . x_r + b1_c > 0] (recomputed from x):
 *   gx   [n, 11] (may be NULL) = go_r s W1^T (w2 o m(r))                 first order, input
 *   d_go [n]     (may be NULL) = s sum_c w2_c m_c(r) (W1[c] . e_r)       second order: the
 *        gradient of (gx . e) w.r.t. go, for the double backward of get_gradient
 *   mlp_grad [PIN_MLP_GRAD_SIZE] += (W1, b1, W2, b2 layout):
 *     flags & PIN_MLP_GRAD_FIRST:  the first-order parameter gradients of sum_r go_r out_r;
 *     flags & PIN_MLP_GRAD_SECOND: the second-order ones, d(sum_r gx_r . e_r)/d params with the
 *       masks held constant: dW1 = s w2 o sum_r m go e^T, dW2 = s W1 . sum_r m go e (b1, b2: 0).
 *   Sums over rows in a fixed order (per-block products on the f32 matrix cores, then one final
 *   reduction).  workspace: pin_mlp_backward_workspace_bytes(n) when flags != 0.
 */
#define PIN_MLP_GRAD_FIRST 1
#define PIN_MLP_GRAD_SECOND 2
int pin_mlp_forward(const PinMlp* mlp, const float* x, int64_t n, float* out, void* stream);
int64_t pin_mlp_backward_workspace_bytes(int64_t n);
int pin_mlp_backward(const PinMlp* mlp, const float* x, int64_t n, const float* go, const float* e, int32_t flags,
                     float* gx, float* d_go, float* mlp_grad, void* workspace, void* stream);

/* pin_train_rows -- coordinates [rows,3] of every row of one iteration (batch + stencil). */
int pin_train_rows(const float* coord, const PinTrainCfg* cfg, float* rows_out, void* stream);

/*
 * pin_train_gather -- Mapper.get_batch's gathers (utils/mapper.py:352-356) fused with the row
 * build: rows_out [rows,3] = every row of the iteration from coord_pool[index] (batch rows, then
 * the stencil of every decimation-th one), label_out [n_main] = label_pool[index], when ts_pool is
 * non-NULL ts_out [n_main] = ts_pool[index], and when weight_pool is non-NULL weight_out [n_main] =
 * |weight_pool[index]| (mapper.py:514).  index: [n_main] int64 pool rows, each in [0, pool_rows):
 * an index outside it is clamped to row 0 and raises bit 0 of *error (device int32, may be NULL;
 * the caller zeroes it and reads it when it wants the check).
 */
int pin_train_gather(const float* coord_pool, const float* label_pool, const int64_t* ts_pool,
                     const float* weight_pool, int64_t pool_rows, const int64_t* index, const PinTrainCfg* cfg,
                     float* rows_out, float* label_out, int64_t* ts_out, float* weight_out, int32_t* error,
                     void* stream);

/*
 * pin_pool_pack -- the sample pool as one 32-B record per sample (8 f32 words): {x, y, z, label,
 * bits(ts lo), bits(ts hi), weight, 0} from coord [n,3], label [n], ts [n] int64 (may be NULL: 0),
 * weight [n] (may be NULL: 1).  packed 16-B aligned, [n, 8] f32.
 * pin_train_gather_packed -- pin_train_gather over such a pool: one line per batch row instead of
 * four (ts_out / weight_out may be NULL: not written; weight_out = |weight|).
 */
int pin_pool_pack(const float* coord, const float* label, const int64_t* ts, const float* weight, int64_t n,
                  float* packed, void* stream);
int pin_train_gather_packed(const float* packed_pool, int64_t pool_rows, const int64_t* index, const PinTrainCfg* cfg,
                            float* rows_out, float* label_out, int64_t* ts_out, float* weight_out, int32_t* error,
                            void* stream);

/* pin_train_gather_packed_split -- pin_train_gather_packed with get_batch's two draws kept apart
 * (utils/mapper.py:335-340): batch rows r < n_index gather pool row index[r], the remaining
 * n_main - n_index rows gather new_idx[index_new[r - n_index]] (new_idx: the new samples' pool rows,
 * new_count of them) -- the torch.cat and the new_idx indexing done by the gather itself.
 * index_new entries outside [0, new_count) are clamped to 0 and reported in *error. */
int pin_train_gather_packed_split(const float* packed_pool, int64_t pool_rows, const int64_t* index, int64_t n_index,
                                  const int64_t* new_idx, int64_t new_count, const int64_t* index_new,
                                  const PinTrainCfg* cfg, float* rows_out, float* label_out, int64_t* ts_out,
                                  float* weight_out, int32_t* error, void* stream);

/* pin_train_gather_packed_draw -- pin_train_gather_packed_split with the batch drawn on the device:
 * get_batch's two torch.randint draws (utils/mapper.py:335-340) replaced by a counter-based
 * generator -- batch row r < n_hist gathers pool row u_r * pool_rows, the rest new_idx[u_r *
 * new_count], u_r = SplitMix64(mix(seed, counter) + r * golden) / 2^64 (a 64 x 64 high multiply).
 * The same (seed, counter) gives the same batch; the caller advances counter per iteration. */
int pin_train_gather_packed_draw(const float* packed_pool, int64_t pool_rows, int64_t n_hist, const int64_t* new_idx,
                                 int64_t new_count, uint64_t seed, uint64_t counter, const PinTrainCfg* cfg,
                                 float* rows_out, float* label_out, int64_t* ts_out, float* weight_out, int32_t* error,
                                 void* stream);

/*
 * pin_train_forward -- training-mode query_feature + Decoder.sdf for every row of one mapping
 * iteration (mapper.py:461-468, :683-711; neural_points.py:528-674 with training_mode): fills
 * st->ids/weights/x/sdf and applies the certainty / ts_update side effects with atomics.
 * Exactly one of hash / grid is non-NULL (grid: non-fat, features read live).
 */
int pin_train_forward(const PinHash* hash, const PinGrid* grid, const PinPoints* pts, const PinMlp* mlp,
                      const float* coord, const int64_t* ts, const PinTrainCfg* cfg, const PinTrainState* st,
                      void* stream);

/* per-block decoder-gradient partial of pin_train_backward: the products T[64][16] and T'[64][16]
 * over the block's rows, then sum so (see k_mlp_grad_final) */
#define PIN_MLP_PART_FLOATS (2 * PIN_HIDDEN_DIM * 16 + 16)

/* Workspace bytes of pin_train_backward for rows = n_main + 6 n_stencil. */
static inline int64_t pin_train_workspace_bytes(int64_t rows) {
    /* a loss double per 64-row wave and a decoder-gradient partial per block, for blocks of
       down to one wave (small batches run one-wave blocks) */
    const int64_t nblk = (rows + 63) / 64;
    return nblk * 8 + nblk * PIN_MLP_PART_FLOATS * 4;
}

/*
 * pin_train_backward -- gradient of  BCEWithLogits(sdf/sigma, sigmoid(label/sigma)) (mean)
 *   + weight_e * mean_k (|g_k| - 1)^2,  g_k = central differences of the stencil rows
 * (mapper.py:515-547) w.r.t. the local features (grad_features [L+1,8] += , may be NULL) and,
 * if mlp_grad != NULL, the decoder parameters (mlp_grad [PIN_MLP_GRAD_SIZE] += , summed in a
 * fixed order).  loss_out (1 double on the device, may be NULL) receives the loss.  workspace:
 * pin_train_workspace_bytes(rows) bytes, needed when loss_out or mlp_grad is non-NULL.
 */
int pin_train_backward(const PinPoints* pts, const PinMlp* mlp, const float* label, const PinTrainCfg* cfg,
                       const PinTrainState* st, float* grad_features, float* mlp_grad, void* workspace,
                       double* loss_out, void* stream);

/* pin_adam_step -- dense Adam over n floats in place (torch.optim.Adam, weight_decay 0). */
int pin_adam_step(float* param, float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, const PinAdamStep* a,
                  void* stream);

/* pin_adam_step_segments -- pin_adam_step over the n feature floats and pin_adam_segments over the
 * decoder's segments in ONE launch, with the same scalars a (a training mapper iteration: the
 * feature and decoder parameter groups of the reference's one optimizer, utils/tools.py:89-116). */
int pin_adam_step_segments(float* param, float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                           float* const* params, const int64_t* sizes, int nseg, float* seg_grad, float* seg_exp_avg,
                           float* seg_exp_avg_sq, const PinAdamStep* a, void* stream);

/*
 * pin_adam_step_train -- one mapper iteration's optimiser step in one launch: the feature step of
 * pin_adam_step (n floats) and, with nseg > 0, the decoder step of pin_adam_segments (whose
 * tensors one block steps).  grad_replicas (replicas > 1, PinTrainState.replica_mode 1): the
 * features' gradient is grad + the sum of the [replicas, n] replicas, which are zeroed again.
 * mlp / packed (non-NULL, nseg > 0): the same block then writes the stepped decoder's
 * pin_mlp_pack image (no pin_mlp_pack call before the next forward).  grad_stride must be 8.
 * grad_fixed (non-NULL; grad_replicas must then be NULL): the deterministic mode's fixed-point
 * replicas of PinTrainState.grad_fixed, [2, max(replicas, 1), n] int64 (coarse part at shift
 * fixed_shift, fine part at fixed_shift + 40): the gradient is grad + float(their integer sums
 * scaled back), and they are zeroed again.
 */
int pin_adam_step_train(float* param, float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                        float* grad_replicas, int32_t replicas, int64_t* grad_fixed, int32_t fixed_shift,
                        float* const* params, const int64_t* sizes, int nseg, float* seg_grad, float* seg_exp_avg,
                        float* seg_exp_avg_sq, const PinMlp* mlp, void* packed, const PinAdamStep* a, void* stream);

/* pin_ref_sort_rows -- test hook for the k-NN tie order (pin_device.h resolve_ties): order[r, :] =
 * the permutation libstdc++'s std::sort leaves row r of keys [rows, n] in (n <= 128), i.e. what the
 * reference's torch.sort(dists2, dim=1) returns as indices (model/neural_points.py:562), computed
 * by the same wave-parallel restatement the query and training kernels use on tied rows. */
int pin_ref_sort_rows(const float* keys, int32_t n, int64_t rows, int32_t* order, void* stream);

/* pin_fixed_accumulate -- out[i] += float((sum_k acc[k n + i]) * 2^-shift) for k < max(nrep, 1),
 * then acc := 0: folds the deterministic mode's fixed-point accumulators (PinTrainState.grad_fixed
 * / cert_fixed) into a float array.  parts 2 (grad_fixed): acc holds a second, fine part of nrep n
 * entries at shift + 40 after the first, added as f64(coarse) 2^-shift + f64(fine) 2^-(shift + 40).
 * The integer sums are exact; the result is rounded once. */
int pin_fixed_accumulate(int64_t* acc, int32_t nrep, int64_t n, int32_t shift, int32_t parts, float* out,
                         void* stream);
/* pin_adam_segments -- the same Adam update over nseg (<= 8) separate parameter tensors params[k]
 * of sizes[k] floats whose gradients and moments lie end to end in contiguous grad / exp_avg /
 * exp_avg_sq (the decoder's W1, b1, W2, b2 against pin_train_backward's mlp_grad): one launch
 * for what torch.optim.Adam does per parameter (utils/tools.py:89-116).  grad_stride must be 8. */
int pin_adam_segments(float* const* params, const int64_t* sizes, int nseg, float* grad, float* exp_avg,
                      float* exp_avg_sq, const PinAdamStep* a, void* stream);

/* pin_adam_rows -- the same Adam update on the listed rows only of [rows, 8] contiguous arrays
 * (param, grad, exp_avg, exp_avg_sq; grad_stride must be 8); those rows' gradients are zeroed
 * when a->zero_grad.  The owned rows of a spatially sharded mapping step (mapper.py shard="space"). */
int pin_adam_rows(float* param, float* grad, float* exp_avg, float* exp_avg_sq, const int64_t* rows, int64_t nrows,
                  const PinAdamStep* a, void* stream);

/* ======================================================================================
 * Map maintenance: insert, local-map selection, prune, pose
 * adjustment and re-hash of NeuralPoints, model/neural_points.py:205-428, with the voxel
 * down-samplers of utils/tools.py:409-477.  Counts that size a caller's allocation are
 * written to DEVICE int64 cells: the caller reads them (one host sync, as the reference's
 * boolean indexing does) -- the calls themselves stay stream-ordered.
 * ====================================================================================== */

/* The per-point arrays of a NeuralPoints map.  Any array but positions may be NULL where a
 * call says so; features has count + 1 rows (the last one is the padding row). */
typedef struct PinMapArrays {
    float* positions;     /* [count,3] f32                 neural_points          */
    float* orientations;  /* [count,4] f32 (w,x,y,z)       point_orientations     */
    int64_t* ts_create;   /* [count]                       point_ts_create        */
    int64_t* ts_update;   /* [count]                       point_ts_update        */
    float* certainties;   /* [count] f32                   point_certainties      */
    float* features;      /* [count+1, feature_dim] f32    geo_features           */
    int64_t count;
    int32_t feature_dim;
    int32_t reserved;
} PinMapArrays;

/* Workspace bytes every map-maintenance call below needs for n elements (points of the frame,
 * or of the map for the whole-map calls). */
int64_t pin_map_workspace_bytes(int64_t n);

/*
 * pin_voxel_down_sample -- one point index per voxel, in ascending order of the reference's
 * flattened voxel key (torch.unique order):
 *   value == NULL: the point closest to its voxel centre after quantising the distance to
 *                  1000 levels, lowest index on ties  (voxel_down_sample_torch, tools.py:409-442)
 *   value != NULL: the point with the smallest quantised value           (tools.py:444-477)
 * Reproduces the key's v_size = grid.max() aliasing (tools.py:430-431), the packed
 * "index + level * 10^digits" amin, and x86 float->int64 conversion of NaN/inf levels.
 * out_idx: [n] int64 (the first *count entries are written); count: 1 device int64.  n >= 1.
 */
int pin_voxel_down_sample(const float* points, int64_t n, float voxel_size, const float* value, int64_t* out_idx,
                          int64_t* count, void* workspace, void* stream);

/*
 * pin_map_insert -- the probe and table write of NeuralPoints.update (neural_points.py:214-242)
 * for the down-sampled points points[sample_idx[i]], i < n:
 *   hash_idx = table[slot];  new = map empty | hash_idx == -1 | |p_hash_idx - p|^2 > dist2_thre
 *          | travel_dist[cur_ts] - travel_dist[ts_update[hash_idx]] > travel_thre;
 *   new points get ids count, count+1, ... in sample order; table[slot] = (new ? id : hash_idx),
 *   the last sample of a shared slot winning (CPU index_put order).
 * new_rows: [n] int64 receives sample_idx[i] of each new point, in id order; n_new: 1 device
 * int64.  positions/ts_update describe the current map (count points).
 */
int pin_map_insert(const float* points, const int64_t* sample_idx, int64_t n, float resolution, int32_t* table,
                   int64_t buffer_size, const float* positions, const int64_t* ts_update, int64_t count,
                   const float* travel_dist, int64_t cur_ts, float dist2_thre, float travel_thre, int64_t* new_rows,
                   int64_t* n_new, void* workspace, void* stream);

/*
 * pin_hash_assign -- table[slot(points[rows[i]])] = rows[i], the last i winning a shared slot
 * (recreate_hash kept_points=True, neural_points.py:405-411).  Leaves other slots alone.
 */
int pin_hash_assign(const float* points, const int64_t* rows, int64_t n, float resolution, int32_t* table,
                    int64_t buffer_size, void* workspace, void* stream);

/*
 * pin_local_map -- local-map selection of reset_local_map (neural_points.py:272-303):
 *   ts_used = use_mid_ts ? long((ts_create + ts_update) / 2) : ts_create;
 *   local = |p - sensor|^2 < radius2 & (use_travel_dist ? |td[cur_ts] - td[ts_used]| < travel_thre
 *                                                       : |cur_ts - ts_used| < diff_ts_local)
 * sensor_position: 3 floats (sensor_f64 = 0) or 3 doubles (sensor_f64 = 1) on the device; the
 * distance test runs in the promoted precision, as torch does for an f64 pose.
 * local_mask [count+1] u8 (last = 1), global2local [count+1] (rank, or g2l_fill off the local
 * map; last = -1), local_rows [count] (global rows of the local points, ascending), local_count
 * (1 device int64).  map needs positions, ts_create (and ts_update when use_mid_ts).
 */
int pin_local_map(const PinMapArrays* map, const float* travel_dist, const void* sensor_position, int32_t sensor_f64,
                  int64_t cur_ts, double radius2, float travel_thre, int32_t use_mid_ts, int32_t use_travel_dist,
                  int64_t diff_ts_local, int64_t g2l_fill, uint8_t* local_mask, int64_t* global2local,
                  int64_t* local_rows, int64_t* local_count, void* workspace, void* stream);

/*
 * pin_prune_rows -- prune_map's selection (neural_points.py:329-337): a point is pruned when
 * |td[cur_ts] - td[ts_update]| > travel_thre and certainty < certainty_thre.  keep_rows [count]
 * receives the kept rows ascending, keep_count (1 device int64) their number.
 */
int pin_prune_rows(const PinMapArrays* map, const float* travel_dist, int64_t cur_ts, float travel_thre,
                   float certainty_thre, int64_t* keep_rows, int64_t* keep_count, void* workspace, void* stream);

/*
 * pin_map_gather -- dst.x[i] = src.x[rows[i]], i < n_rows, for every array non-NULL in dst
 * (boolean-mask / index selection of reset_local_map :293-309, prune_map :339-349 and
 * recreate_hash :414-421).  pad_row != 0 also copies the features padding row:
 * dst.features[n_rows] = src.features[src.count].  dst.count is not read.  A negative row
 * index writes zeros (gather) or is skipped (scatter).
 */
int pin_map_gather(const PinMapArrays* src, const int64_t* rows, int64_t n_rows, int32_t pad_row,
                   const PinMapArrays* dst, void* stream);

/*
 * pin_pool_window -- the training pool's window filter (utils/mapper.py:226-262):
 * keep[0..k) = the rows i < n (ascending) with sum((coord[i] - center)^2) < radius2, counts[0] = k,
 * counts[1] = the kept rows with i >= tail_start (the current frame's samples, :256-259).
 * center: 3 values on the device, double when center_f64 (then the arithmetic is f64, as torch
 * promotes an f32 pool minus an f64 pose), else float (f32 arithmetic, radius2 rounded to f32);
 * the sum in the reference's order.  One host read of counts sizes what follows.
 * workspace: pin_pool_window_workspace_bytes(n).
 */
int64_t pin_pool_window_workspace_bytes(int64_t n);
int pin_pool_window(const float* coord, int64_t n, const void* center, int32_t center_f64, double radius2,
                    int64_t tail_start, int64_t* keep, int64_t* counts, void* workspace, void* stream);

/* One array of a multi-array row gather: row i of dst = row rows[i] of src, row_bytes each. */
typedef struct PinRowArray {
    const void* src;
    void* dst;
    int64_t row_bytes;
} PinRowArray;
#define PIN_ROW_ARRAYS_MAX 8

/*
 * pin_gather_rows -- for every array a < n_arrays (<= PIN_ROW_ARRAYS_MAX):
 * a.dst[i] = a.src[rows[i]] (row_bytes bytes), i < n_rows, all arrays in one launch; each row
 * moves with the widest of 16/8/4/1-byte accesses its size and both pointers allow.  The training
 * pool's window filter (utils/mapper.py:226-262: the index selection of coord, global coord,
 * label, weight, ts and the packed records by one kept-row list) -- torch.index_select per pool
 * in the reference.  rows must be in [0, source rows); dst must not overlap src.
 */
int pin_gather_rows(const PinRowArray* arrays, int32_t n_arrays, const int64_t* rows, int64_t n_rows, void* stream);

/*
 * pin_map_scatter -- dst.x[rows[i]] = src.x[i] for every array non-NULL in src (assign_local_to_
 * global, neural_points.py:315-324); pad_row != 0 also writes src.features[n_rows] to
 * dst.features[dst.count].
 */
int pin_map_scatter(const PinMapArrays* src, const int64_t* rows, int64_t n_rows, int32_t pad_row,
                    const PinMapArrays* dst, void* stream);

/*
 * pin_map_adjust -- adjust_map (neural_points.py:355-370) in place: each point moves by the
 * pose correction pose_diff[ts_used] ([T,4,4] f32 row-major; ts_used as in pin_local_map):
 * p = R p + t, q = quat(R) * q (utils/tools.py:326-334, :356-369, :401-407).
 */
int pin_map_adjust(const PinMapArrays* map, const float* pose_diff, int64_t num_poses, int32_t use_mid_ts,
                   void* stream);

/* ---------------------------------------------------------------------------------------
 * Training samples along the scan rays (utils/data_sampler.py:20-192) + pose transform
 * (utils/mapper.py:133-215 via transform_torch, utils/tools.py:386-399).
 * Scalars that the reference evaluates in Python double before touching a tensor are passed
 * pre-rounded to f32. */
typedef struct PinSampleCfg {
    int32_t surface_n, front_n, behind_n;  /* surface_sample_n, free_front_n, free_behind_n */
    float surface_range;         /* surface_sample_range_m */
    float two_range;             /* f32(2.0 * surface_sample_range_m)  (sigma_ratio * range) */
    float front_min_ratio;       /* free_sample_begin_ratio */
    float end_dist;              /* free_sample_end_dist_m */
    int32_t dist_weight_on;      /* weight = dist_weight_base - (d / max_range) * dist_weight_scale */
    float dist_weight_base;      /* f32(1 + dist_weight_scale * 0.5) */
    float dist_weight_scale;
    float max_range;
    int32_t behind_dropoff_on;   /* weight *= clamp((dropoff_max - disp) / dropoff_diff, 0, 1) * 0.8 + 0.2 */
    float dropoff_max;           /* free_sample_end_dist_m */
    float dropoff_diff;          /* f32(end - 0.2 * end) */
    const float* pose;           /* [4,4] row-major f32 sensor pose (device), read if global_coord */
} PinSampleCfg;

/*
 * pin_sample_rays -- DataSampler.sample (utils/data_sampler.py:20-192) for n rays (points in the
 * sensor frame): writes n * (1 + surface_n + front_n + behind_n) rows in the reference's ray-wise
 * order: coord [rows,3] (sensor frame), sdf_label [rows], weight [rows] (negative = free space),
 * and, if global_coord != NULL, transform_torch(coord, pose) [rows,3].  randn_surface [surface_n*n],
 * rand_front [front_n*n], rand_behind [behind_n*n] are the reference's draws (torch.randn /
 * torch.rand, part-major).
 */
int pin_sample_rays(const float* points, int64_t n, const float* randn_surface, const float* rand_front,
                    const float* rand_behind, const PinSampleCfg* cfg, float* coord, float* sdf_label, float* weight,
                    float* global_coord, void* stream);

/*
 * pin_deskew -- deskewing (utils/tools.py:540-567) in place: rows of `stride` floats whose first
 * three are x, y, z; ts [n] point times, ts_minmax [2] = (min, max) of ts (device, e.g.
 * torch.aminmax); pose [4,4] row-major f32 (T_last<-cur).  s = (ts - min) / (max - min) -
 * ts_mid_pose; p <- exp(s log R) p + s t  (roma.rotmat_slerp(I, R, s), Rodrigues in f32).
 */
int pin_deskew(float* points, int64_t n, int64_t stride, const float* ts, const float* ts_minmax, const float* pose,
               float ts_mid_pose, void* stream);

/* ---------------------------------------------------------------------------------------
 * Marching cubes for Mesher.mc_mesh (utils/mesher.py:310-337; the reference calls
 * skimage.measure.marching_cubes(sdf, level=0, allow_degenerate=False, mask=mc_mask)).
 * values [nx][ny][nz] f32 (x slowest); mask [nx][ny][nz] u8 or NULL: cube (x,y,z) -- grid points
 * x..x+1, y..y+1, z..z+1 -- is processed iff mask[x][y][z].  Triangles from the table of
 * tools/gen_mc_table.py; one vertex per used grid edge at the linear crossing, in index space;
 * right-hand normals point from values < level to values >= level.  Two calls: pin_mc_count
 * writes counts[2] = {vertices, faces} (device) and leaves the vertex / face numbering in the
 * workspace; pin_mc_emit (same arguments and workspace) writes verts [V,3] f32 and faces [F,3]
 * int32 in cube order.  nx*ny*nz < 2^29. */
int64_t pin_mc_workspace_bytes(int64_t nx, int64_t ny, int64_t nz);
int pin_mc_count(const float* values, const uint8_t* mask, int64_t nx, int64_t ny, int64_t nz, float level,
                 void* workspace, int64_t* counts, void* stream);
int pin_mc_emit(const float* values, int64_t nx, int64_t ny, int64_t nz, float level, const void* workspace,
                float* verts, int32_t* faces, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PIN_SLAM_AMD_H */
