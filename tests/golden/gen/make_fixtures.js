// Fixture generator — runs ONLY in the build container, where /root/reference exists.
//
// It executes the reference's OWN JavaScript (vendored babylon.js 5.0.0-alpha.43, the glTF
// loader, BVH_Fast_Builder.js and the unmodified *_Path_Tracing.js setup scripts) under Node with
// a recording stand-in for the Babylon effect API (EffectWrapper / EffectRenderer /
// RenderTargetTexture / RawTexture / Texture), and writes what crosses that boundary:
//   * every render call per frame (effect, target, uniforms set through effect.set*, samplers),
//   * the Float32Array payloads handed to RawTexture.CreateRGBATexture (BVH + triangle textures).
// Nothing from the reference is copied into the repository; only these numeric outputs are kept
// (tests/golden/*.npz / *.json, packed by make_fixtures.py).
//
// usage: node make_fixtures.js <scene> <outdir> [width height frames seed model]
//   scene: cornell | gltf | sky | hdri | quadric
//   model: a menu name, or file:<model file>:<modelInitialScale>:<rh 0|1> (mesh payloads only)
'use strict';
const fs = require('fs');
const path = require('path');
const vm = require('vm');

const REF = process.env.PT_REFERENCE || '/root/reference';
const [scene, outdir, W_, H_, F_, SEED_, MODEL_] = process.argv.slice(2);
const W = parseInt(W_ || '256', 10), H = parseInt(H_ || '256', 10);
const FRAMES = parseInt(F_ || '4', 10);
const SEED = BigInt(SEED_ || '1');
const MODEL = MODEL_ || 'Stanford Bunny';
fs.mkdirSync(outdir, { recursive: true });

const ENV = require('./browser_env.js');
const { REAL, BABYLON } = ENV.setup(REF, W, H, SEED);

// ---------------------------------------------------------------- recording boundary
let renderLoop = null;
const RealNull = REAL.NullEngine;
class RecEngine extends RealNull {
  constructor() { super({ renderWidth: W, renderHeight: H, textureSize: 512, deterministicLockstep: false, lockstepMaxSteps: 1 }); this.isPointerLock = false; }
  runRenderLoop(f) { renderLoop = f; }
  enterPointerlock() {}
  getDeltaTime() { return 1000 / 60; }
  setHardwareScalingLevel() {}
  resize() {}
}
BABYLON.Engine = RecEngine;

const rawTextures = [];
class RecRT {
  constructor(name, size) { this.name = name; this._w = size.width; this._h = size.height; }
  getSize() { return { width: this._w, height: this._h }; }
  resize(s) { this._w = s.width; this._h = s.height; }
}
BABYLON.RenderTargetTexture = RecRT;
class RecTexture {
  constructor(url, scene, noMipmap, invertY, sampling, onLoad) {
    this.name = 'file:' + String(url).replace(/^.*\//, '');
    this.noMipmap = noMipmap; this.invertY = invertY; this.sampling = sampling;
    this._hdr = /\.hdr$/i.test(String(url));
    // the .hdr environments are missing from the reference: the loader "decodes" the synthetic one
    if (this._hdr && onLoad) setImmediate(onLoad);
  }
  getSize() { return this._hdr ? { width: ENV.HDR_W, height: ENV.HDR_H } : { width: 1, height: 1 }; }
  readPixels() { return Promise.resolve(this._hdr ? ENV.syntheticHDR() : new Float32Array(4)); }
}
BABYLON.Texture = RecTexture;
BABYLON.RawTexture = {
  CreateRGBATexture(data, w, h, scn, mips, invertY, sampling, type) {
    const t = { name: 'raw' + rawTextures.length, w, h, invertY, sampling, type, data: Float32Array.from(data) };
    rawTextures.push(t);
    return t;
  },
};

let frames = [];
let current = null;
function texName(t) { return t === null || t === undefined ? null : (t.name || '?'); }
class RecEffect {
  constructor(wrapper) { this.wrapper = wrapper; }
  _u(n, v) { current.uniforms[n] = v; }
  setTexture(n, t) { current.samplers[n] = texName(t); }
  setFloat(n, v) { this._u(n, ['f', [v]]); }
  setFloat2(n, a, b) { this._u(n, ['f', [a, b]]); }
  setFloat3(n, a, b, c) { this._u(n, ['f', [a, b, c]]); }
  setVector3(n, v) { this._u(n, ['f', [v.x, v.y, v.z]]); }
  setInt(n, v) { this._u(n, ['i', [v]]); }
  setBool(n, v) { this._u(n, ['i', [v ? 1 : 0]]); }
  setMatrix(n, m) { this._u(n, ['f', Array.from(m.m !== undefined ? m.m : m.toArray())]); }
}
class RecWrapper {
  constructor(o) {
    this.name = o.name; this.uniformNames = o.uniformNames; this.samplerNames = o.samplerNames;
    this.effect = new RecEffect(this); this._obs = [];
    this.onApplyObservable = { add: (f) => this._obs.push(f) };
    this.fragmentShaderKey = Object.keys(BABYLON.Effect.ShadersStore).find((k) => BABYLON.Effect.ShadersStore[k] === o.fragmentShader) || null;
  }
}
BABYLON.EffectWrapper = RecWrapper;
BABYLON.EffectRenderer = class { constructor() {} render(w, target) {
  current = { effect: w.name, shader: w.fragmentShaderKey, target: texName(target), uniforms: {}, samplers: {} };
  w._obs.forEach((f) => f());
  frames[frames.length - 1].push(current);
} };

// ---------------------------------------------------------------- run the reference scripts
function runScript(rel) { vm.runInThisContext(fs.readFileSync(path.join(REF, rel), 'utf8'), { filename: rel }); }
const scripts = {
  cornell: ['js/PathTracingCommon.js', 'js/BabylonPathTracing_FragmentShader.js', 'js/Babylon_Path_Tracing.js'],
  sky: ['js/PathTracingCommon.js', 'js/PhysicalSkyModel_FragmentShader.js', 'js/Physical_Sky_Model.js'],
  gltf: ['js/PathTracingCommon.js', 'js/GLTFModelPathTracing_FragmentShader.js', 'js/BVH_Fast_Builder.js', 'js/GLTF_Model_Path_Tracing.js'],
  hdri: ['js/PathTracingCommon.js', 'js/HDRIEnvironmentPathTracing_FragmentShader.js', 'js/BVH_Fast_Builder.js', 'js/HDRI_Environment_Path_Tracing.js'],
  quadric: ['js/PathTracingCommon.js', 'js/TransformedQuadricGeometry_FragmentShader.js', 'js/Transformed_Quadric_Geometry.js'],
};
// the setup scripts resolve models/ and textures/ relative to the page: make them absolute file URLs
const realLoad = REAL.SceneLoader.LoadAssetContainer.bind(REAL.SceneLoader);
BABYLON.SceneLoader = Object.assign(Object.create(REAL.SceneLoader), { LoadAssetContainer: (root, file, ...rest) => realLoad('file://' + path.join(REF, root) + '/', file, ...rest) });

const tick = () => new Promise((r) => setImmediate(r));
function frame() { frames.push([]); renderLoop(); }

// the BVH builder's own input (per-triangle AABB min/max/centroid, js/GLTF_Model_Path_Tracing.js:
// 421-454), captured as BVH_Build_Iterative receives it: the native builder is pinned against it
let builderInput = null;
function wrapBuilder() {
  const real = vm.runInThisContext('BVH_Build_Iterative');
  globalThis.BVH_Build_Iterative = function (workList, aabb) {
    builderInput = { work: Uint32Array.from(workList), aabb: Float32Array.from(aabb.subarray(0, 9 * workList.length)) };
    return real(workList, aabb);
  };
}

(async () => {
  for (const s of scripts[scene]) { runScript(s); if (s.endsWith('BVH_Fast_Builder.js')) wrapBuilder(); }
  const meshTextures = () => rawTextures.filter((t) => t.h === 2048);
  const hdrTextures = () => rawTextures.filter((t) => t.h !== 2048);
  if (scene === 'gltf' || scene === 'hdri') {
    // wait for the initial (teapot) load (and the environment), then select MODEL through the GUI
    // exactly as a user would
    while (meshTextures().length < 2 || (scene === 'hdri' && hdrTextures().length < 1)) { frame(); await tick(); }
    if (MODEL.startsWith('file:')) {
      // a model file outside the menu (file:<name>:<modelInitialScale>:<rh 0|1>): set what the
      // menu handler sets and call the script's own loadModel()
      const [, file, scale, rh] = MODEL.split(':');
      const before = meshTextures().length;
      vm.runInThisContext(`modelNameAndExtension = ${JSON.stringify(file)}; modelWasDefinedInRHCoordSystem = ${rh === '1'};` +
                          ` modelInitialScale = ${Number(scale)}; loadModel();`);
      while (meshTextures().length < before + 2) { frame(); await tick(); }
    } else if (MODEL !== 'Utah Teapot') {
      const before = meshTextures().length;
      vm.runInThisContext('gltfModel_SelectionController').setValue(MODEL);
      while (meshTextures().length < before + 2) { frame(); await tick(); }
    }
    // GUI-triggered changes (scale/rotation controllers) restart accumulation within a few frames:
    // start the recording at the last restart (uFrameCounter == 1)
    frames = [];
    for (let i = 0; i < 6; i++) frame();
    const fc = (f) => f[0].uniforms.uFrameCounter[1][0];
    let start = frames.length - 1;
    while (start > 0 && fc(frames[start]) !== 1) start--;
    frames = frames.slice(start);
  } else {
    frames = [];
  }
  // recorded frames: the uniform stream the setup script pushes from here on. PT_CONTROLS (JSON,
  // one entry per recorded frame) drives the script's own input state before that frame, as its
  // event handlers would: {down: [key names], up: [...], wheel: +1|-1, rot: [pitch, yaw]}
  // (KeyboardState via onKeyDown/onKeyUp, increaseFOV/decreaseFOV via onMouseWheel, and
  // camera.rotation as the pointer-lock mouse input leaves it)
  const controls = process.env.PT_CONTROLS ? JSON.parse(process.env.PT_CONTROLS) : null;
  const applyControls = (c) => {
    if (!c) return;
    const ks = vm.runInThisContext('KeyboardState');
    for (const k of c.down || []) ks[k] = true;
    for (const k of c.up || []) ks[k] = false;
    if (c.wheel > 0) vm.runInThisContext('increaseFOV = true');
    if (c.wheel < 0) vm.runInThisContext('decreaseFOV = true');
    if (c.rot) vm.runInThisContext('camera').rotation.set(c.rot[0], c.rot[1], 0);
  };
  while (frames.length < FRAMES) { if (controls) applyControls(controls[frames.length]); frame(); }
  frames = frames.slice(0, FRAMES);
  const hasMesh = scene === 'gltf' || scene === 'hdri';
  const meta = { scene, width: W, height: H, seed: Number(SEED), model: hasMesh ? MODEL : null, frames };
  if (controls) meta.controls = controls;
  if (hasMesh) {
    const tris = vm.runInThisContext('total_number_of_triangles');
    const mt = meshTextures(), n = mt.length;
    const aabb = mt[n - 2], tri = mt[n - 1];
    const nodes = 2 * tris - 1;
    fs.writeFileSync(path.join(outdir, 'bvh.f32'), Buffer.from(aabb.data.buffer, 0, nodes * 8 * 4));
    fs.writeFileSync(path.join(outdir, 'tri.f32'), Buffer.from(tri.data.buffer, 0, tris * 32 * 4));
    if (!builderInput || builderInput.work.length !== tris) throw new Error('builder input not captured');
    for (let i = 0; i < tris; i++) if (builderInput.work[i] !== i) throw new Error('unexpected work list');
    fs.writeFileSync(path.join(outdir, 'aabb_in.f32'), Buffer.from(builderInput.aabb.buffer));
    meta.triangles = tris; meta.nodes = nodes;
    meta.textures = { [aabb.name]: 'bvh', [tri.name]: 'tri' };
    meta.modelScale = vm.runInThisContext('modelInitialScale');
  }
  if (scene === 'hdri') {
    const ht = hdrTextures(), env = ht[ht.length - 1];
    meta.textures[env.name] = 'hdr';
    meta.hdr = { width: env.w, height: env.h, invertY: env.invertY, sampling: env.sampling === undefined ? null : env.sampling,
                 generator: 'synthetic_hdr v1', sha256: require('crypto').createHash('sha256').update(Buffer.from(env.data.buffer)).digest('hex') };
  }
  fs.writeFileSync(path.join(outdir, 'frames.json'), JSON.stringify(meta));
  process.stdout.write(`ok ${scene} ${W}x${H} frames=${FRAMES}\n`);
})().catch((e) => { console.error(e); process.exit(1); });
