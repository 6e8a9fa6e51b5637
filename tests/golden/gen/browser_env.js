// browser_env.js — the browser-ish globals the reference's page scripts expect, for running them
// under Node (test infrastructure, build container only): seeded Math.random, window/document/
// navigator stubs, Stats and dat.GUI stand-ins, a local-file XMLHttpRequest, and a writable facade
// over the vendored babylon.js module. Used by make_fixtures.js (recording boundary) and by
// tests/js/dropin_check.js (the product's babylon_pt.js shim over a mock addon).
'use strict';
const fs = require('fs');
const path = require('path');
const Module = require('module');

function setup(REF, W, H, SEED) {
  // ---------------------------------------------------------------- deterministic Math.random
  // splitmix64 -> top 24 bits / 2^24 (exactly representable in fp32, so the uniform is lossless)
  let smState = BigInt(SEED);
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


  return { REAL, BABYLON };
}

// Synthetic equirect environment (the reference's .hdr files are not in the repository it ships):
// a float RGBA image whose every value is a short dyadic rational, so the same bits come out of
// Float32Array here and of tests/helpers.py synthetic_hdr(): a bright-top sky gradient, a dark
// ground, 8-bit hashed noise, and a 5x5 sun whose centre texel is the unique brightest value
// (the setup script derives uSunDirection from it, js/HDRI_Environment_Path_Tracing.js:774-815).
const HDR_W = 2048, HDR_H = 1024, SUN_X = 1536, SUN_Y = 300;
function hash32(i) {
  let h = Math.imul(i, 0x9E3779B1) >>> 0;
  h = (h ^ (h >>> 15)) >>> 0;
  h = Math.imul(h, 0x85EBCA77) >>> 0;
  return (h ^ (h >>> 13)) >>> 0;
}
function syntheticHDR() {
  const d = new Float32Array(HDR_W * HDR_H * 4);
  for (let y = 0; y < HDR_H; y++) {
    for (let x = 0; x < HDR_W; x++) {
      const i = y * HDR_W + x;
      const n = (hash32(i) & 255) / 4096;
      let r, g, b;
      if (y < HDR_H / 2) { const t = (HDR_H / 2 - y) / 2048; r = 0.25 + t + n; g = 0.375 + t + n; b = 0.75 + 2 * t + n; }
      else { r = 0.125 + n; g = 0.1875 + n; b = 0.0625 + n; }
      const dx = x - SUN_X, dy = y - SUN_Y;
      if (dx >= -2 && dx <= 2 && dy >= -2 && dy <= 2) { r = g = b = (dx === 0 && dy === 0) ? 4096 : 512; }
      d[4 * i] = r; d[4 * i + 1] = g; d[4 * i + 2] = b; d[4 * i + 3] = 1;
    }
  }
  return d;
}

module.exports = { setup, syntheticHDR, HDR_W, HDR_H };
