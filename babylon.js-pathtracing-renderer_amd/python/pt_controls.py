"""The demos' interactive render loop, restated for the Python host.

What one iteration of the setup scripts' ``engine.runRenderLoop`` callback computes before it
renders (js/Babylon_Path_Tracing.js:374-604 == js/GLTF_Model_Path_Tracing.js:1063-1227, the same
block in every demo): elapsed time, a fresh ``uRandomVec2``, camera-moved detection by comparing
the camera world matrix with last frame's, WASD/QE flight along the camera basis, ``-``/``=``
focus distance, ``[``/``]`` aperture, mouse-wheel FOV in 1 degree steps, and the progressive
counters (``uFrameCounter``, ``uSampleCounter``, ``uOneOverSampleCounter``, ``uCameraIsMoving``).
The uniforms it produces drive :class:`babylon_pt.StreamPlayer` (``play_call(call, uniforms)``)
or any EffectWrapper directly.

The camera is Babylon's UniversalCamera (vendored js/babylon.js, 5.0.0-alpha.43) on the path the
demos use (no parent, left-handed scene, Euler rotation with zero roll): world matrix =
invert(LookAtLH(position, position + R·(0,0,1), up)), R from RotationYawPitchRoll. It is restated
operation by operation - JS doubles, rounded to float32 wherever Babylon stores into a Matrix's
Float32Array - so ``uCameraMatrix`` matches the reference bit for bit (pinned by
tests/golden/controls_cornell.json, the Cornell script run under Node with its own input state
driven; tests/test_controls.py). Mouse-look itself (Babylon's FreeCameraMouseInput) is not
restated: set ``camera.rotation`` as the pointer-lock input would leave it.
"""
import math

import numpy as np

__all__ = ["UniversalCamera", "RenderLoop", "KEYS"]

# the key names the scripts test (KEYCODE_NAMES values, js/Babylon_Path_Tracing.js:110-124)
KEYS = ("w", "a", "s", "d", "q", "e", "dash", "equals", "leftbracket", "rightbracket")


def _f32(x):
    return float(np.float32(x))


def _normalize(v):
    """Vector3.normalize (normalizeFromLength: lengths 0 and 1 leave the vector unchanged)."""
    n = math.sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2])
    if n == 0 or n == 1:
        return list(v)
    s = 1 / n
    return [v[0] * s, v[1] * s, v[2] * s]


def _cross(l, r):
    return [l[1] * r[2] - l[2] * r[1], l[2] * r[0] - l[0] * r[2], l[0] * r[1] - l[1] * r[0]]


def _dot(l, r):
    return l[0] * r[0] + l[1] * r[1] + l[2] * r[2]


def rotation_yaw_pitch_roll(yaw, pitch, roll):
    """Matrix.RotationYawPitchRollToRef: Quaternion.RotationYawPitchRollToRef then
    Matrix.FromQuaternionToRef (float32 storage)."""
    r, o, a = 0.5 * roll, 0.5 * pitch, 0.5 * yaw
    s, c = math.sin(r), math.cos(r)
    l, u = math.sin(o), math.cos(o)
    h, d = math.sin(a), math.cos(a)
    x = d * l * c + h * u * s
    y = h * u * c - d * l * s
    z = d * u * s - h * l * c
    w = d * u * c + h * l * s
    xx, yy, zz = x * x, y * y, z * z
    xy, zw, zx, yw, yz, xw = x * y, z * w, z * x, y * w, y * z, x * w
    m = [1 - 2 * (yy + zz), 2 * (xy + zw), 2 * (zx - yw), 0,
         2 * (xy - zw), 1 - 2 * (zz + xx), 2 * (yz + xw), 0,
         2 * (zx + yw), 2 * (yz - xw), 1 - 2 * (yy + xx), 0,
         0, 0, 0, 1]
    return [_f32(v) for v in m]


def look_at_lh(eye, target, up):
    """Matrix.LookAtLHToRef (float32 storage)."""
    s = _normalize([target[0] - eye[0], target[1] - eye[1], target[2] - eye[2]])
    o = _cross(up, s)
    c = o[0] * o[0] + o[1] * o[1] + o[2] * o[2]
    if c == 0:
        o[0] = 1
    else:
        n = math.sqrt(c)
        if n != 1:
            k = 1 / n
            o = [o[0] * k, o[1] * k, o[2] * k]
    a = _normalize(_cross(s, o))
    m = [o[0], a[0], s[0], 0, o[1], a[1], s[1], 0, o[2], a[2], s[2], 0,
         -_dot(o, eye), -_dot(a, eye), -_dot(s, eye), 1]
    return [_f32(v) for v in m]


def invert(mm):
    """Matrix.invertToRef: cofactor expansion in doubles over the float32 entries, float32 out
    (a singular matrix is returned unchanged, as Babylon copies it)."""
    n, r, o, a, s, c, l, u, h, d, p, f, _, mz, g, v = mm
    y = p * v - g * f
    b = d * v - mz * f
    T = d * g - mz * p
    E = h * v - _ * f
    S = h * g - p * _
    R = h * mz - _ * d
    A = +(c * y - l * b + u * T)
    x = -(s * y - l * E + u * S)
    P = +(s * b - c * E + u * R)
    C = -(s * T - c * S + l * R)
    O = n * A + r * x + o * P + a * C
    if O == 0:
        return list(mm)
    M = 1 / O
    I = l * v - g * u
    D = c * v - mz * u
    N = c * g - mz * l
    L = s * v - _ * u
    w = s * g - _ * l
    F = s * mz - _ * c
    B = l * f - p * u
    U = c * f - d * u
    V = c * p - d * l
    k = s * f - h * u
    G = s * p - h * l
    z = s * d - h * c
    j = -(r * y - o * b + a * T)
    W = +(n * y - o * E + a * S)
    H = -(n * b - r * E + a * R)
    X = +(n * T - r * S + o * R)
    Y = +(r * I - o * D + a * N)
    K = -(n * I - o * L + a * w)
    Q = +(n * D - r * L + a * F)
    q = -(n * N - r * w + o * F)
    Z = -(r * B - o * U + a * V)
    J = +(n * B - o * k + a * G)
    dd = -(n * U - r * k + a * z)
    ee = +(n * V - r * G + o * z)
    out = [A * M, j * M, Y * M, Z * M, x * M, W * M, K * M, J * M,
           P * M, H * M, Q * M, dd * M, C * M, X * M, q * M, ee * M]
    return [_f32(t) for t in out]


class UniversalCamera:
    """Babylon's UniversalCamera on the demos' path: ``position`` and ``rotation`` (pitch, yaw,
    roll = 0) in JS doubles, ``fov`` in radians (Babylon's default 0.8)."""

    def __init__(self, position, rotation=(0.0, 0.0, 0.0), fov=0.8):
        self.position = [float(v) for v in position]
        self.rotation = [float(v) for v in rotation]
        self.fov = float(fov)
        self.up = [0.0, 1.0, 0.0]

    def world_matrix(self):
        """TargetCamera._getViewMatrix + Camera.getViewMatrix's invertToRef: 16 float32 values
        (column-major, as uCameraMatrix)."""
        if self.rotation[2] != 0:
            raise ValueError("camera roll is not on the demos' path (the up vector would rotate)")
        rm = rotation_yaw_pitch_roll(self.rotation[1], self.rotation[0], self.rotation[2])
        # Vector3.TransformCoordinatesToRef(_referencePoint (0,0,1), rm): w = 1
        ref = [0 * rm[0] + 0 * rm[4] + 1 * rm[8] + rm[12],
               0 * rm[1] + 0 * rm[5] + 1 * rm[9] + rm[13],
               0 * rm[2] + 0 * rm[6] + 1 * rm[10] + rm[14]]
        wi = 1 / (0 * rm[3] + 0 * rm[7] + 1 * rm[11] + rm[15])
        ref = [ref[0] * wi, ref[1] * wi, ref[2] * wi]
        p = self.position
        target = [p[0] + ref[0], p[1] + ref[1], p[2] + ref[2]]
        return invert(look_at_lh(p, target, self.up))


class RenderLoop:
    """One demo's render loop state. ``step()`` runs one iteration and returns the uniforms it
    sets that frame (the effect's ``["f"|"i", [values]]`` form, ready for
    ``StreamPlayer.play_call(call, uniform_override=...)``).

    Input (what the scripts' DOM handlers set): ``key_down(name)`` / ``key_up(name)`` with the
    names in :data:`KEYS`, ``wheel(delta_y)`` (> 0 widens the FOV), ``resize(w, h)``,
    ``invalidate()`` for a GUI change that restarts accumulation (the ``needChange*`` flags).
    ``random`` returns the next Math.random() value (default: Python's ``random.random``).
    Defaults are the Cornell / glTF demos' (js/Babylon_Path_Tracing.js:242-250)."""

    def __init__(self, width, height, camera=None, cam_flight_speed=100.0, aperture=0.0, focus_distance=113.0,
                 aperture_step=1.0, focus_step=1.0, scene_is_dynamic=False, delta_ms=1000 / 60, random=None):
        if random is None:
            import random as _r
            random = _r.random
        self.width, self.height = int(width), int(height)
        self.camera = camera or UniversalCamera((0.0, -20.0, -120.0))
        self.cam_flight_speed = float(cam_flight_speed)
        self.aperture = float(aperture)
        self.focus_distance = float(focus_distance)
        self.aperture_step = float(aperture_step)
        self.focus_step = float(focus_step)
        self.scene_is_dynamic = bool(scene_is_dynamic)
        self.delta_ms = float(delta_ms)           # engine.getDeltaTime()
        self.random = random
        self.keys = set()
        self.time = 0.0                           # timeInSeconds
        self.frame_counter = 1.0                  # uFrameCounter (1: it seeds the shader's rng)
        self.sample_counter = 0.0                 # uSampleCounter
        self.camera_recently_moving = False
        self.old_matrix = [0.0] * 16              # oldCameraMatrix = new BABYLON.Matrix() (zeros)
        self._increase_fov = self._decrease_fov = False
        self._resized = False
        self._invalid = False

    # ---- input (the scripts' event handlers)
    def key_down(self, name):
        if name not in KEYS:
            raise ValueError("unknown key %r (one of %s)" % (name, ", ".join(KEYS)))
        self.keys.add(name)

    def key_up(self, name):
        self.keys.discard(name)

    def wheel(self, delta_y):
        if delta_y > 0:
            self._increase_fov = True
        elif delta_y < 0:
            self._decrease_fov = True

    def resize(self, width, height):
        self.width, self.height = int(width), int(height)
        self._resized = True

    def invalidate(self):
        self._invalid = True

    def _pressed(self, k, other):
        return k in self.keys and other not in self.keys

    # ---- one iteration
    def step(self):
        moving = self._invalid or self._resized
        self._invalid = self._resized = False
        self.time += self.delta_ms * 0.001
        frame_time = self.delta_ms * 0.001
        rv = (self.random(), self.random())

        nm = self.camera.world_matrix()           # getWorldMatrix() at the top of the frame
        if nm != self.old_matrix:
            moving = True
        self.old_matrix = nm
        fwd = _normalize(nm[8:11])
        up = _normalize(nm[4:7])
        right = _normalize(nm[0:3])
        step = self.cam_flight_speed * frame_time
        pos = self.camera.position

        def move(v, sign):
            sv = [v[0] * step, v[1] * step, v[2] * step]
            for i in range(3):
                pos[i] = pos[i] + sv[i] if sign > 0 else pos[i] - sv[i]

        if self._pressed("w", "s"):
            move(fwd, +1)
        if self._pressed("s", "w"):
            move(fwd, -1)
        if self._pressed("a", "d"):
            move(right, -1)
        if self._pressed("d", "a"):
            move(right, +1)
        if self._pressed("e", "q"):
            move(up, +1)
        if self._pressed("q", "e"):
            move(up, -1)
        if self._pressed("equals", "dash"):
            self.focus_distance += self.focus_step
            moving = True
        if self._pressed("dash", "equals"):
            self.focus_distance -= self.focus_step
            if self.focus_distance < 1:
                self.focus_distance = 1.0
            moving = True
        if self._pressed("rightbracket", "leftbracket"):
            self.aperture += self.aperture_step
            if self.aperture > 100000.0:
                self.aperture = 100000.0
            moving = True
        if self._pressed("leftbracket", "rightbracket"):
            self.aperture -= self.aperture_step
            if self.aperture < 0.0:
                self.aperture = 0.0
            moving = True
        if self._increase_fov:
            self.camera.fov += math.pi / 180
            if self.camera.fov > 150 * (math.pi / 180):
                self.camera.fov = 150 * (math.pi / 180)
            moving = True
            self._increase_fov = False
        if self._decrease_fov:
            self.camera.fov -= math.pi / 180
            if self.camera.fov < 1 * (math.pi / 180):
                self.camera.fov = 1 * (math.pi / 180)
            moving = True
            self._decrease_fov = False

        if not moving:
            self.sample_counter = 1.0 if self.scene_is_dynamic else self.sample_counter + 1.0
            self.frame_counter += 1.0
            self.camera_recently_moving = False
        else:
            self.sample_counter = 1.0
            self.frame_counter += 1.0
            if not self.camera_recently_moving:
                self.frame_counter = 1.0
                self.camera_recently_moving = True

        vlen = math.tan(self.camera.fov * 0.5)
        ulen = vlen * (self.width / self.height)
        # pathTracingScene.render() recomputes the camera before the effect's onApply reads it
        cam = self.camera.world_matrix()
        return {
            "uResolution": ["f", [float(self.width), float(self.height)]],
            "uRandomVec2": ["f", [rv[0], rv[1]]],
            "uULen": ["f", [ulen]],
            "uVLen": ["f", [vlen]],
            "uTime": ["f", [self.time]],
            "uFrameCounter": ["f", [self.frame_counter]],
            "uSampleCounter": ["f", [self.sample_counter]],
            "uApertureSize": ["f", [self.aperture]],
            "uFocusDistance": ["f", [self.focus_distance]],
            "uCameraIsMoving": ["i", [1 if moving else 0]],
            "uCameraMatrix": ["f", cam],
            "uOneOverSampleCounter": ["f", [1.0 / self.sample_counter]],
        }
