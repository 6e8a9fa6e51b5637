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
//   scene: cornell | gltf | sky
'use strict';
const fs = require('fs');
const path = require('path');
const vm = require('vm');
const Module = require('module');

const REF = process.env.PT_REFERENCE || '/root/reference';
const [scene, outdir, W_, H_, F_, SEED_, MODEL_] = process.argv.slice(2);
const W = parseInt(W_ || '256', 10), H = parseInt(H_ || '256', 10);
const FRAMES = parseInt(F_ || '4', 10);
const SEED = BigInt(SEED_ || '1');
const MODEL = MODEL_ || 'Stanford Bunny';
fs.mkdirSync(outdir, { recursive: true });

// ---------------------------------------------------------------- deterministic Math.random
// splitmix64 -> top 24 bits / 2^24 (exactly representable in fp32, so the uniform is lossless)
let smState = SEED;
function splitmix64() {
  smState = (smState + 0x9E3779B97F4A7C15n) & 0xFFFFFFFFFFFFFFFFn;
  let z = smState;
  z = ((z ^ (z >> 30n)) * 0xBF58476D1CE4E5B9n) & 0xFFFFFFFFFFFFFFFFn;
  z = ((z ^ (z >> 27n)) * 0x94D049BB133111EBn) & 0xFFFFFFFFFFFFFFFFn;
  return z ^ (z >> 31n);
}
Math.random = () => Number(splitmix64() >> 40n) / 16777216;

// ---------------------------------------------------------------- browser-ish globals
global.window = global; global.self = global;
global.navigator = { userAgent: 'node', maxTouchPoints: 0 };
global.atob = (s) => Buffer.from(s, 'base64').toString('binary');
global.btoa = (s) => Buffer.from(s, 'binary').toString('base64');
function fakeElement() {
  return { style: {}, innerHTML: '', addEventListener() {}, removeEventListener() {}, appendChild() {},
           getBoundingClientRect() { return { left: 0, top: 0, width: W, height: H }; },
           focus() {}, setAttribute() {}, getContext() { return null; }, width: W, height: H };
}
global.document = { getElementById: () => fakeElement(), addEventListener() {}, removeEventListener() {},
                    createElement: () => fakeElement(), body: fakeElement() };
global.addEventListener = () => {};
global.removeEventListener = () => {};
global.Stats = function () { this.domElement = fakeElement(); this.update = () => {}; };
function Controller(obj, prop) { this.object = obj; this.property = prop; this.__onChange = null; }
Controller.prototype.onChange = function (f) { this.__onChange = f; return this; };
Controller.prototype.onFinishChange = function () { return this; };
Controller.prototype.getValue = function () { return this.object[this.property]; };
Controller.prototype.setValue = function (v) { this.object[this.property] = v; if (this.__onChange) this.__onChange.call(this, v); return this; };
Controller.prototype.name = function () { return this; };
Controller.prototype.step = function () { return this; };
function GUI() {}
GUI.prototype.add = function (obj, prop) { return new Controller(obj, prop); };
GUI.prototype.addColor = GUI.prototype.add;
GUI.prototype.addFolder = function () { return new GUI(); };
GUI.prototype.open = GUI.prototype.close = function () {};
global.dat = { GUI };

// local-file XMLHttpRequest (the glTF loader fetches through it)
class LocalXHR {
  constructor() { this.readyState = 0; this.status = 0; this._l = {}; this.responseType = ''; this.onreadystatechange = null; }
  open(m, url) { this._url = url; this.readyState = 1; }
  setRequestHeader() {} getResponseHeader() { return null; } getAllResponseHeaders() { return ''; } abort() {}
  addEventListener(e, f) { (this._l[e] = this._l[e] || []).push(f); }
  removeEventListener(e, f) { if (this._l[e]) this._l[e] = this._l[e].filter((g) => g !== f); }
  send() {
    const p = decodeURIComponent(this._url.replace(/^file:\/\//, '').split('?')[0]);
    setImmediate(() => {
      try {
        const b = fs.readFileSync(p);
        this.status = 200;
        if (this.responseType === 'arraybuffer') this.response = b.buffer.slice(b.byteOffset, b.byteOffset + b.byteLength);
        else { this.response = b.toString('utf8'); this.responseText = this.response; }
      } catch (e) { this.status = 404; this.response = null; }
      this.readyState = 4;
      if (this.onreadystatechange) this.onreadystatechange();
      for (const ev of ['readystatechange', 'load', 'loadend']) (this._l[ev] || []).forEach((f) => f.call(this));
    });
  }
}
global.XMLHttpRequest = LocalXHR;

const origResolve = Module._resolveFilename;
Module._resolveFilename = function (req, ...rest) {
  if (req === 'babylonjs') return path.join(REF, 'js/babylon.js');
  return origResolve.call(this, req, ...rest);
};
const REAL = require(path.join(REF, 'js/babylon.js'));
// a writable facade over the module namespace (its exports are getter-only)
const BABYLON = {};
for (const k of Object.keys(REAL)) {
  Object.defineProperty(BABYLON, k, { configurable: true, enumerable: true, get: () => REAL[k],
    set: (v) => Object.defineProperty(BABYLON, k, { value: v, writable: true, configurable: true, enumerable: true }) });
}
global.BABYLON = BABYLON;
require(path.join(REF, 'js/babylon.glTFFileLoader.min.js'));
BABYLON.Logger.LogLevels = BABYLON.Logger.ErrorLogLevel;

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
  constructor(url, scene, noMipmap, invertY, sampling) {
    this.name = 'file:' + String(url).replace(/^.*\//, '');
    this.noMipmap = noMipmap; this.invertY = invertY; this.sampling = sampling;
  }
  readPixels() { return Promise.resolve(new Float32Array(4)); }
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
};
// the setup scripts resolve models/ and textures/ relative to the page: make them absolute file URLs
const realLoad = REAL.SceneLoader.LoadAssetContainer.bind(REAL.SceneLoader);
BABYLON.SceneLoader = Object.assign(Object.create(REAL.SceneLoader), { LoadAssetContainer: (root, file, ...rest) => realLoad('file://' + path.join(REF, root) + '/', file, ...rest) });

const tick = () => new Promise((r) => setImmediate(r));
function frame() { frames.push([]); renderLoop(); }

(async () => {
  for (const s of scripts[scene]) runScript(s);
  if (scene === 'gltf') {
    // wait for the initial (teapot) load, then select MODEL through the GUI exactly as a user would
    while (rawTextures.length < 2) { frame(); await tick(); }
    if (MODEL !== 'Utah Teapot') {
      const before = rawTextures.length;
      vm.runInThisContext('gltfModel_SelectionController').setValue(MODEL);
      while (rawTextures.length < before + 2) { frame(); await tick(); }
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
  // recorded frames: the uniform stream the setup script pushes from here on
  while (frames.length < FRAMES) frame();
  frames = frames.slice(0, FRAMES);
  const meta = { scene, width: W, height: H, seed: Number(SEED), model: scene === 'gltf' ? MODEL : null, frames };
  if (scene === 'gltf') {
    const tris = vm.runInThisContext('total_number_of_triangles');
    const n = rawTextures.length;
    const aabb = rawTextures[n - 2], tri = rawTextures[n - 1];
    const nodes = 2 * tris - 1;
    fs.writeFileSync(path.join(outdir, 'bvh.f32'), Buffer.from(aabb.data.buffer, 0, nodes * 8 * 4));
    fs.writeFileSync(path.join(outdir, 'tri.f32'), Buffer.from(tri.data.buffer, 0, tris * 32 * 4));
    meta.triangles = tris; meta.nodes = nodes;
    meta.textures = { [aabb.name]: 'bvh', [tri.name]: 'tri' };
    meta.modelScale = vm.runInThisContext('modelInitialScale');
  }
  fs.writeFileSync(path.join(outdir, 'frames.json'), JSON.stringify(meta));
  process.stdout.write(`ok ${scene} ${W}x${H} frames=${FRAMES}\n`);
})().catch((e) => { console.error(e); process.exit(1); });
