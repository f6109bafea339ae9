"""The glm operations the reference's scenes use, with glm's semantics.

nim-glm-fork (nim.cfg:1) is not vendored, so these follow the standard GLM
definitions (column-major Mat4x4, post-multiplying translate/rotate). KAT 2 of
SURVEY.md 8(c) (test/boxtest.nim:32-33) pins X-axis rotate + translate +
Mat4*Vec4; everything else here is "parity unpinned" beyond GLM's published
formulas. Matrices are numpy float64 arrays of shape (4, 4) indexed m[col][row]
exactly like glm, so m.reshape(16) is the column-major ABI layout.
"""
import math

import numpy as np

X_AXIS = np.array([1.0, 0.0, 0.0])  # geom.nim:7
Y_AXIS = np.array([0.0, 1.0, 0.0])  # geom.nim:8
Z_AXIS = np.array([0.0, 0.0, 1.0])  # geom.nim:9

RadPerDeg = math.pi / 180.0


def degToRad(d):
    """Nim math.degToRad: d * (PI / 180)."""
    return float(d) * RadPerDeg


def mat4(diag=1.0):
    return np.eye(4, dtype=np.float64) * float(diag)


def vec(x, y, z):
    """geom.nim:11 — direction, w = 0."""
    return np.array([x, y, z, 0.0], dtype=np.float64)


def point(x, y, z):
    """geom.nim:14 — position, w = 1."""
    return np.array([x, y, z, 1.0], dtype=np.float64)


def vec3(x, y=None, z=None):
    if y is None:
        y = z = x
    return np.array([x, y, z], dtype=np.float64)


def dot(a, b):
    r = 0.0
    for i in range(len(a)):
        r = r + float(a[i]) * float(b[i])
    return r


def normalize(v):
    """v / length(v), component count preserved (vec4 normalize keeps w = 0)."""
    v = np.asarray(v, dtype=np.float64)
    ln = math.sqrt(dot(v, v))
    return np.array([float(c) / ln for c in v], dtype=np.float64)


def translate(m, v):
    """glm translate: m * T(v); Result[3] = m[0]*v0 + m[1]*v1 + m[2]*v2 + m[3]."""
    m = np.asarray(m, dtype=np.float64)
    r = m.copy()
    r[3] = m[0] * v[0] + m[1] * v[1] + m[2] * v[2] + m[3]
    return r


def rotate(m, axis_or_angle, angle_or_axis):
    """glm rotate: m * R(axis, angle) (Rodrigues form of GLM's matrix_transform).

    Accepts both argument orders used by the reference scenes:
    m.rotate(X_AXIS, degToRad(-12.0)).
    """
    if np.ndim(axis_or_angle) == 0:
        angle, axis = float(axis_or_angle), angle_or_axis
    else:
        axis, angle = axis_or_angle, float(angle_or_axis)
    m = np.asarray(m, dtype=np.float64)
    c = math.cos(angle)
    s = math.sin(angle)
    ax = normalize(np.asarray(axis, dtype=np.float64)[:3])
    temp = (1.0 - c) * ax
    R = np.zeros((3, 3))
    R[0][0] = c + temp[0] * ax[0]
    R[0][1] = temp[0] * ax[1] + s * ax[2]
    R[0][2] = temp[0] * ax[2] - s * ax[1]
    R[1][0] = temp[1] * ax[0] - s * ax[2]
    R[1][1] = c + temp[1] * ax[1]
    R[1][2] = temp[1] * ax[2] + s * ax[0]
    R[2][0] = temp[2] * ax[0] + s * ax[1]
    R[2][1] = temp[2] * ax[1] - s * ax[0]
    R[2][2] = c + temp[2] * ax[2]
    r = np.zeros((4, 4))
    r[0] = m[0] * R[0][0] + m[1] * R[0][1] + m[2] * R[0][2]
    r[1] = m[0] * R[1][0] + m[1] * R[1][1] + m[2] * R[1][2]
    r[2] = m[0] * R[2][0] + m[1] * R[2][1] + m[2] * R[2][2]
    r[3] = m[3]
    return r


def scale(m, v):
    m = np.asarray(m, dtype=np.float64)
    r = m.copy()
    r[0] = m[0] * v[0]
    r[1] = m[1] * v[1]
    r[2] = m[2] * v[2]
    return r


def inverse(m):
    """GLM compute_inverse for mat4 (cofactor form, times 1/determinant).

    The same algorithm is exported natively as rt_mat4_inverse (rtmi.h).
    """
    m = np.asarray(m, dtype=np.float64)
    Coef00 = m[2][2] * m[3][3] - m[3][2] * m[2][3]
    Coef02 = m[1][2] * m[3][3] - m[3][2] * m[1][3]
    Coef03 = m[1][2] * m[2][3] - m[2][2] * m[1][3]
    Coef04 = m[2][1] * m[3][3] - m[3][1] * m[2][3]
    Coef06 = m[1][1] * m[3][3] - m[3][1] * m[1][3]
    Coef07 = m[1][1] * m[2][3] - m[2][1] * m[1][3]
    Coef08 = m[2][1] * m[3][2] - m[3][1] * m[2][2]
    Coef10 = m[1][1] * m[3][2] - m[3][1] * m[1][2]
    Coef11 = m[1][1] * m[2][2] - m[2][1] * m[1][2]
    Coef12 = m[2][0] * m[3][3] - m[3][0] * m[2][3]
    Coef14 = m[1][0] * m[3][3] - m[3][0] * m[1][3]
    Coef15 = m[1][0] * m[2][3] - m[2][0] * m[1][3]
    Coef16 = m[2][0] * m[3][2] - m[3][0] * m[2][2]
    Coef18 = m[1][0] * m[3][2] - m[3][0] * m[1][2]
    Coef19 = m[1][0] * m[2][2] - m[2][0] * m[1][2]
    Coef20 = m[2][0] * m[3][1] - m[3][0] * m[2][1]
    Coef22 = m[1][0] * m[3][1] - m[3][0] * m[1][1]
    Coef23 = m[1][0] * m[2][1] - m[2][0] * m[1][1]
    Fac0 = np.array([Coef00, Coef00, Coef02, Coef03])
    Fac1 = np.array([Coef04, Coef04, Coef06, Coef07])
    Fac2 = np.array([Coef08, Coef08, Coef10, Coef11])
    Fac3 = np.array([Coef12, Coef12, Coef14, Coef15])
    Fac4 = np.array([Coef16, Coef16, Coef18, Coef19])
    Fac5 = np.array([Coef20, Coef20, Coef22, Coef23])
    Vec0 = np.array([m[1][0], m[0][0], m[0][0], m[0][0]])
    Vec1 = np.array([m[1][1], m[0][1], m[0][1], m[0][1]])
    Vec2 = np.array([m[1][2], m[0][2], m[0][2], m[0][2]])
    Vec3 = np.array([m[1][3], m[0][3], m[0][3], m[0][3]])
    Inv0 = Vec1 * Fac0 - Vec2 * Fac1 + Vec3 * Fac2
    Inv1 = Vec0 * Fac0 - Vec2 * Fac3 + Vec3 * Fac4
    Inv2 = Vec0 * Fac1 - Vec1 * Fac3 + Vec3 * Fac5
    Inv3 = Vec0 * Fac2 - Vec1 * Fac4 + Vec2 * Fac5
    SignA = np.array([+1.0, -1.0, +1.0, -1.0])
    SignB = np.array([-1.0, +1.0, -1.0, +1.0])
    inv = np.array([Inv0 * SignA, Inv1 * SignB, Inv2 * SignA, Inv3 * SignB])
    Row0 = np.array([inv[0][0], inv[1][0], inv[2][0], inv[3][0]])
    Dot0 = m[0] * Row0
    Dot1 = (Dot0[0] + Dot0[1]) + (Dot0[2] + Dot0[3])
    if Dot1 == 0.0:
        raise ValueError("singular matrix")
    one_over_det = 1.0 / Dot1
    return inv * one_over_det


def mul(m, v):
    """Mat4 * Vec4: sum of columns scaled by v, accumulated from zero."""
    m = np.asarray(m, dtype=np.float64)
    r = np.zeros(4)
    for c in range(4):
        r = r + m[c] * v[c]
    return r


def flat(m):
    """Column-major 16-double ABI layout."""
    return np.ascontiguousarray(np.asarray(m, dtype=np.float64).reshape(16))
