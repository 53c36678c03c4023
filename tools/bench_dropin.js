"use strict";
// Drop-in throughput leg of bench.py (value_dropin): drives a gossip-shaped workload through the
// JS IBlsVerifier (lodestar_amd/js/index.js) exactly as Lodestar's gossip validators call it --
// one verifySignatureSets(sets, {batchable: true}) per job, keys as registered index2pubkey
// handles -- and times first submission -> last promise settled, so JS marshalling (packJobs),
// the pinned-buffer copy, H2D, every kernel and D2H are inside the timed region.  Each round is
// timed on its own; the line reports the median round (>= 10 rounds, as the reference's
// .benchrc.yaml minRuns), the GPU_MAX_HW_QUEUES the HIP runtime runs with, and the latency of a
// 1-set verifyOnMainThread call (a gossip block's proposer check, validation/block.ts:143-146)
// issued while a round of gossip batches is in flight: its promise's settle time (the loop is
// busy submitting the round meanwhile), the part of the call that runs on the loop (blocked), and
// the synchronous entry's device latency on the same engine.
//   node tools/bench_dropin.js <workload.bin> <engines> <rounds>
// workload.bin (little-endian, written by bench.py): u32 magic 0x4C424430, n_keys, n_jobs, n_sets,
// n_pks, slots; then keys (n_keys x 96 B), job_off (n_jobs+1 u32), pk_off (n_sets+1 u32),
// pk_idx (n_pks u32, indices into keys), roots (n_sets x 32 B), sigs (n_sets x 96 B), and the
// expected per-job verdict (n_jobs i32).
const fs = require("fs");
const path = require("path");
const m = require(path.join(__dirname, "..", "lodestar_amd", "js", "index.js"));

async function main() {
  const [file, enginesArg, roundsArg] = process.argv.slice(2);
  const buf = fs.readFileSync(file);
  const u32 = (off) => buf.readUInt32LE(off);
  if (u32(0) !== 0x4c424430) throw Error("bad workload file");
  const nKeys = u32(4), nJobs = u32(8), nSets = u32(12), nPks = u32(16), slots = u32(20);
  let off = 24;
  const take = (bytes) => {
    const v = new Uint8Array(buf.buffer, buf.byteOffset + off, bytes);
    off += bytes;
    return v;
  };
  const takeU32 = (n) => {
    const v = new Uint32Array(n);
    for (let i = 0; i < n; i++) v[i] = buf.readUInt32LE(off + 4 * i);
    off += 4 * n;
    return v;
  };
  const keys = take(nKeys * 96);
  const jobOff = takeU32(nJobs + 1);
  const pkOff = takeU32(nSets + 1);
  const pkIdx = takeU32(nPks);
  const roots = take(nSets * 32);
  const sigs = take(nSets * 96);
  const expected = takeU32(nJobs);
  const engines = Number(enginesArg || 4), rounds = Math.max(Number(roundsArg || 10), 1);

  const pool = new m.BlsGpuVerifier({engines});
  const handles = pool.registerPubkeys(Array.from({length: nKeys}, (_, k) => keys.subarray(96 * k, 96 * k + 96)));
  // the ISignatureSet objects the gossip validators would hold (built outside the timed region)
  const jobs = [];
  for (let j = 0; j < nJobs; j++) {
    const sets = [];
    for (let i = jobOff[j]; i < jobOff[j + 1]; i++) {
      const pks = [];
      for (let q = pkOff[i]; q < pkOff[i + 1]; q++) pks.push(handles[pkIdx[q]]);
      sets.push({type: "aggregate", pubkeys: pks, signingRoot: roots.subarray(32 * i, 32 * i + 32),
                 signature: sigs.subarray(96 * i, 96 * i + 96)});
    }
    jobs.push(sets);
  }
  const perSlot = Math.ceil(nJobs / slots);
  async function round() {
    const ps = [];
    for (let s = 0; s < slots; s++) {
      for (let j = s * perSlot; j < Math.min(nJobs, (s + 1) * perSlot); j++)
        ps.push(pool.verifySignatureSets(jobs[j], {batchable: true}));
      await new Promise((r) => setImmediate(r));  // gossip arrives slot by slot
    }
    return Promise.all(ps);
  }
  const warm = await round();
  warm.forEach((v, j) => {
    if (v !== (expected[j] === 1)) throw Error(`job ${j}: ${v} != expected ${expected[j]}`);
  });
  const per = [];
  const t0 = process.hrtime.bigint();
  for (let r = 0; r < rounds; r++) {
    const r0 = process.hrtime.bigint();
    await round();
    per.push(Number(process.hrtime.bigint() - r0) / 1e9);
  }
  const el = Number(process.hrtime.bigint() - t0) / 1e9;
  const sorted = per.slice().sort((a, b) => a - b);
  const med = sorted[Math.floor(sorted.length / 2)];
  const stats = Object.assign({}, pool.stats);
  // verifyOnMainThread (its own engine) while a round of gossip is in flight on the pool's engines
  const one = [{type: "aggregate", pubkeys: [handles[pkIdx[0]]], signingRoot: roots.subarray(0, 32),
                signature: sigs.subarray(0, 96)}];
  // blocked: the part of the call that runs on the event loop (the call returns its promise at
  // once; the reference's synchronous blst verify blocks for the whole verification)
  const lat = [];
  const blocked = [];
  for (let k = 0; k < 10; k++) {
    const bg = round();
    await new Promise((r) => setImmediate(r));
    const c0 = process.hrtime.bigint();
    const p = pool.verifySignatureSets(one, {verifyOnMainThread: true});
    blocked.push(Number(process.hrtime.bigint() - c0) / 1e6);
    const ok = await p;
    lat.push(Number(process.hrtime.bigint() - c0) / 1e6);
    if (ok !== (expected[0] === 1)) throw Error("main-thread verdict");
    await bg;
  }
  lat.sort((a, b) => a - b);
  blocked.sort((a, b) => a - b);
  // the same 1-set call through the synchronous entry (verifySignatureSet: the device latency on
  // the latency engine, blocking the loop as the reference's verifyOnMainThread does): separates
  // the device's latency under the pool's load from the event loop's queueing of the promise
  const latSync = [];
  for (let k = 0; k < 10; k++) {
    const bg = round();
    await new Promise((r) => setImmediate(r));
    const c0 = process.hrtime.bigint();
    const ok = pool.verifySignatureSet(one[0]);
    latSync.push(Number(process.hrtime.bigint() - c0) / 1e6);
    if (ok !== (expected[0] === 1)) throw Error("main-thread verdict (sync)");
    await bg;
  }
  latSync.sort((a, b) => a - b);
  await pool.close();
  console.log(JSON.stringify({value_dropin: Math.round(nSets / med), value_dropin_mean: Math.round((nSets * rounds) / el),
                              seconds: Number(el.toFixed(3)), rounds, round_s_median: Number(med.toFixed(4)),
                              engines, gpu_max_hw_queues: m.addon.hwQueues(), sets_per_round: nSets,
                              batches: stats.batches, mean_sets_per_batch: Math.round(stats.sets / Math.max(stats.batches, 1)),
                              // the synchronous entry: the device latency under the pool's load, the
                              // quantity round 5 reported under this name (its verifyOnMainThread was
                              // synchronous)
                              main_thread_1set_ms_under_load: Number(latSync[Math.floor(latSync.length / 2)].toFixed(3)),
                              // verifyOnMainThread since round 6: the promise's settle time (includes the
                              // event loop's queueing behind the round's own submissions) and the part of
                              // the call that runs on the loop
                              verify_on_main_thread_promise_ms_under_load: Number(lat[Math.floor(lat.length / 2)].toFixed(3)),
                              main_thread_1set_blocked_ms: Number(blocked[Math.floor(blocked.length / 2)].toFixed(3)),
                              main_thread_1set_blocked_ms_max: Number(blocked[blocked.length - 1].toFixed(3))}));
}

main().catch((e) => {
  console.error(e);
  process.exit(1);
});
