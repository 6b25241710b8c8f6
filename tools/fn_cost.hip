// fn_cost.hip -- dynamic instruction cost of each device function on the solver path.
//
// One kernel per function, each lane applying the function once to inputs drawn
// like the solver's own (unit quaternions with w >= 0, angles in [0, pi], arm
// vectors, 3- and 5-point Kabsch fits).  Run under
//   rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU ... -- tools/fn_cost
// and subtract the `empty` kernel: the difference is the per-wave (= per-call,
// one call per lane) VALU / SALU / f64 count of the function.  It also prints
// throughput (ps per call, chip-wide) from HIP events.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt
//         -fno-fast-math -I include -I humanoid-real-time-retarget_amd/csrc tools/fn_cost.hip -o tools/fn_cost
#include <cstdio>

#include <cstdlib>

#include "rtg_math.cuh"

using namespace rtg;

#define NLANES (1 << 21)

__device__ __forceinline__ float u01(uint32_t i, uint32_t k)
{
    uint32_t h = i * 0x9E3779B1u ^ (k * 0x85EBCA77u + 0x165667B1u);
    h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12; h *= 0x297A2D39u; h ^= h >> 15;
    return (float)(h >> 8) * (1.0f / 16777216.0f);
}
__device__ __forceinline__ float sn(uint32_t i, uint32_t k) { return 2.0f * u01(i, k) - 1.0f; }
__device__ __forceinline__ Q rq(uint32_t i) { return qnormalize(Q{sn(i, 1), sn(i, 2), sn(i, 3), sn(i, 4)}); }
__device__ __forceinline__ V rv(uint32_t i, uint32_t k) { return V{sn(i, k), sn(i, k + 1), sn(i, k + 2)}; }

enum {
    F_EMPTY, F_EXP, F_ACOS, F_SINCOS, F_ATAN2, F_NORMANG, F_RADB, F_FAA, F_QNORM, F_ROTMAT, F_KAB3, F_KAB5,
    F_EULER, F_QXYZ, F_SHPR, F_ELPY, F_QROT, F_DIV, F_EXPTAB, F_QMULNORM, F_HANDX, F_SQRTCR, F_SCRCP, F_RCP64,
    F_QXYZF, F_GESDD3, F_LARTG, F_LASV2, F_LARFG2, F_COUNT
};
static const char *kNames[F_COUNT] = {"empty", "qexp_component", "cr_acos", "cr_sincos", "f_atan2f",
                                      "normalize_angle", "radians_between", "qfrom_angle_axis", "qnormalize",
                                      "qfrom_rotmat", "cal_joint_quat<3>", "cal_joint_quat<5>", "scipy_as_euler",
                                      "quat_in_xyz_axis", "shoulder_pr", "elbow_py", "qrotate", "f32 div",
                                      "exp_dof (table)", "qmul_norm", "hand_x_mean", "cr_sqrt", "sqrt_clamp_rcp",
                                      "rcp64+mulr_q", "quat_in_xyz_intrinsic",
                                      "la_gesdd3 (5-pt A)", "la_lartg", "la_lasv2", "la_larfg<2>"};

template <int F>
__global__ __launch_bounds__(256) void kcost(float *out, const uint32_t *__restrict__ tab)
{
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    float r = 0.0f;
    if (F == F_EMPTY) {
        const Q q = rq(i);
        r = q.x + q.w;
    } else if (F == F_EXP) {
        r = qexp_component(rq(i), 1);
    } else if (F == F_ACOS) {
        r = cr_acos(rq(i).w);
    } else if (F == F_SINCOS) {
        const SC t = cr_sincos((double)(3.14159265f * rq(i).w));
        r = t.s + t.c;
    } else if (F == F_ATAN2) {
        const Q q = rq(i);
        r = f_atan2f(q.x, q.w);
    } else if (F == F_NORMANG) {
        r = normalize_angle(3.14159265f * rq(i).w);
    } else if (F == F_RADB) {
        r = radians_between(rv(i, 1), rv(i, 4), rv(i, 7));
    } else if (F == F_FAA) {
        const Q q = qfrom_angle_axis(3.0f * sn(i, 9), V{0.f, 1.f, 0.f});
        r = q.y + q.w;
    } else if (F == F_QNORM) {
        const Q q = qnormalize(Q{sn(i, 1), sn(i, 2), sn(i, 3), sn(i, 4)});
        r = q.x + q.w;
    } else if (F == F_ROTMAT) {
        const Q q0 = rq(i);
        const float m[9] = {1 - 2 * (q0.y * q0.y + q0.z * q0.z), 2 * (q0.x * q0.y - q0.w * q0.z),
                            2 * (q0.x * q0.z + q0.w * q0.y),     2 * (q0.x * q0.y + q0.w * q0.z),
                            1 - 2 * (q0.x * q0.x + q0.z * q0.z), 2 * (q0.y * q0.z - q0.w * q0.x),
                            2 * (q0.x * q0.z - q0.w * q0.y),     2 * (q0.y * q0.z + q0.w * q0.x),
                            1 - 2 * (q0.x * q0.x + q0.y * q0.y)};
        const Q q = qfrom_rotmat(m);
        r = q.x + q.w;
    } else if (F == F_KAB3) {
        const Q q0 = rq(i);
        const V Z[3] = {V{0.1f, 0.02f, 0.3f}, V{-0.2f, 0.1f, 0.05f}, V{0.05f, -0.3f, 0.1f}};
        V M[3];
        for (int k = 0; k < 3; ++k) {
            const V v = qrotate(q0, Z[k]);
            M[k] = V{v.x + 0.002f * sn(i, 20 + k), v.y + 0.002f * sn(i, 30 + k), v.z};
        }
        const Q q = cal_joint_quat<3>(Z, M);
        r = q.x + q.w;
    } else if (F == F_KAB5) {
        const Q q0 = rq(i);
        const V Z[5] = {V{0.1f, 0.02f, 0.03f}, V{0.12f, 0.01f, 0.0f}, V{0.11f, -0.01f, -0.02f},
                        V{0.1f, -0.03f, -0.03f}, V{0.03f, 0.04f, 0.02f}};
        V M[5];
        for (int k = 0; k < 5; ++k) {
            const V v = qrotate(q0, Z[k]);
            M[k] = V{v.x + 0.002f * sn(i, 20 + k), v.y + 0.002f * sn(i, 30 + k), v.z};
        }
        const Q q = cal_joint_quat<5>(Z, M);
        r = q.x + q.w;
    } else if (F == F_EULER) {
        double a[3];
        scipy_as_euler(rq(i), 0, 1, 2, false, a);
        r = (float)(a[0] + a[1] + a[2]);
    } else if (F == F_QXYZ) {
        Q e[3];
        quat_in_xyz_axis(rq(i), 0, 1, 2, false, e);
        r = e[0].x + e[1].y + e[2].z;
    } else if (F == F_SHPR) {
        Q p, rr;
        shoulder_pr(rv(i, 1), ArmZero{0.3f, -0.2f}, rq(i), p, rr);
        r = p.y + rr.x;
    } else if (F == F_ELPY) {
        Q y, e;
        elbow_py(rv(i, 1), ArmZero{0.3f, -0.2f}, rq(i), y, e);
        r = y.z + e.y;
    } else if (F == F_QROT) {
        const V v = qrotate(rq(i), rv(i, 5));
        r = v.x + v.y + v.z;
    } else if (F == F_DIV) {
        const Q q = rq(i);
        r = q.x / q.w;
    } else if (F == F_EXPTAB) {   // one exp-map DOF read-out through the angle table (all entries tabulated)
        const Q q = rq(i);
        r = exp_dof_finish(exp_dof_table_part(q.w, tab), q.y);
    } else if (F == F_QMULNORM) {
        const Q q = qmul_norm(rq(i), rq(i + 7));
        r = q.x + q.w;
    } else if (F == F_HANDX) {
        const V tip[5] = {rv(i, 3), rv(i, 6), rv(i, 9), rv(i, 12), rv(i, 15)};
        const Q rot = rq(i);   // rtg_solver.cuh hand_x_mean
        const float x0 = qrotate(rot, rv(i, 18)).x;
        r = mean5(qrotate(rot, tip[0]).x - x0, qrotate(rot, tip[1]).x - x0, qrotate(rot, tip[2]).x - x0,
                  qrotate(rot, tip[3]).x - x0, qrotate(rot, tip[4]).x - x0);
    } else if (F == F_SQRTCR) {
        r = cr_sqrt(rq(i).w + 1.5f);
    } else if (F == F_SCRCP) {
        const NormRcp n = sqrt_clamp_rcp(rq(i).w + 1.5f, 1e-9f);
        r = n.n + (float)n.r.r;
    } else if (F == F_QXYZF) {   // the solvers' 'XYZ' split (round 5: atan2-free, scipy fallback)
        Q e[3];
        quat_in_xyz_intrinsic(rq(i), e);
        r = e[0].x + e[1].y + e[2].z;
    } else if (F == F_GESDD3) {   // the SVD alone on a wrist-fit-like A (column-major)
        const Q q0 = rq(i);
        const V Z[5] = {V{0.1f, 0.02f, 0.03f}, V{0.12f, 0.01f, 0.0f}, V{0.11f, -0.01f, -0.02f},
                        V{0.1f, -0.03f, -0.03f}, V{0.03f, 0.04f, 0.02f}};
        float a[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        for (int k = 0; k < 5; ++k) {
            const V v = qrotate(q0, Z[k]);
            const V m{v.x + 0.002f * sn(i, 20 + k), v.y + 0.002f * sn(i, 30 + k), v.z};
            a[0] += m.x * Z[k].x; a[3] += m.x * Z[k].y; a[6] += m.x * Z[k].z;
            a[1] += m.y * Z[k].x; a[4] += m.y * Z[k].y; a[7] += m.y * Z[k].z;
            a[2] += m.z * Z[k].x; a[5] += m.z * Z[k].y; a[8] += m.z * Z[k].z;
        }
        Svd3 z;
        la_gesdd3(a, z);
        r = z.u[0] + z.vt[4];
    } else if (F == F_LARTG) {
        float c, sv, rr;
        la_lartg(sn(i, 1), sn(i, 2), c, sv, rr);
        r = c + sv + rr;
    } else if (F == F_LASV2) {
        float a0, a1, a2, a3, a4, a5;
        la_lasv2(sn(i, 1), sn(i, 2), sn(i, 3), a0, a1, a2, a3, a4, a5);
        r = a0 + a1 + a2 + a3 + a4 + a5;
    } else if (F == F_LARFG2) {
        float al = sn(i, 1), x0 = sn(i, 2), x1 = sn(i, 3);
        const float tau = la_larfg<2>(al, x0, x1);
        r = tau + al + x0 + x1;
    } else if (F == F_RCP64) {
        const Q q = rq(i);
        const Q u = mulr_q(q, rcp64(q.w + 2.0f));
        r = u.x + u.y + u.z + u.w;
    }
    out[i] = r;
}

static const uint32_t *g_tab;
template <int F>
static float run(float *d)
{
    hipEvent_t s, e;
    (void)hipEventCreate(&s);
    (void)hipEventCreate(&e);
    hipLaunchKernelGGL(kcost<F>, dim3(NLANES / 256), dim3(256), 0, 0, d, g_tab);
    (void)hipEventRecord(s);
    const int reps = 5;
    for (int k = 0; k < reps; ++k) hipLaunchKernelGGL(kcost<F>, dim3(NLANES / 256), dim3(256), 0, 0, d, g_tab);
    (void)hipEventRecord(e);
    (void)hipEventSynchronize(e);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, s, e);
    return ms / reps;
}

template <int F>
static void all(float *d, float *t)
{
    t[F] = run<F>(d);
    if constexpr (F + 1 < F_COUNT) all<F + 1>(d, t);
}

int main()
{
    float *d;
    if (hipMalloc(&d, NLANES * sizeof(float)) != hipSuccess) return 1;
    uint32_t *tab;   // every code 4: the table path with move 0 for every w in [0.25, 1)
    if (hipMalloc(&tab, kAngTabWords * sizeof(uint32_t)) != hipSuccess) return 1;
    if (hipMemset(tab, 0, kAngTabWords * sizeof(uint32_t)) != hipSuccess) return 1;
    {
        uint32_t *h = (uint32_t *)malloc(kAngTabWords * sizeof(uint32_t));
        for (uint32_t k = 0; k < kAngTabWords; ++k) h[k] = 0x24924924u;   // 3-bit codes 4,4,... (10 per word)
        if (hipMemcpy(tab, h, kAngTabWords * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess) return 1;
        free(h);
    }
    g_tab = tab;
    float t[F_COUNT];
    all<0>(d, t);
    printf("%-22s %10s %12s\n", "function", "us/2^21", "ps/call net");
    for (int k = 0; k < F_COUNT; ++k) printf("%-22s %10.2f %12.3f\n", kNames[k], t[k] * 1e3, (t[k] - t[0]) * 1e9 / NLANES);
    (void)hipFree(d);
    return 0;
}
