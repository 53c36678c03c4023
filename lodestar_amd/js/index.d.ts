// Type declarations for the MI355X IBlsVerifier drop-in (lodestar_amd/js/index.js).
// Mirrors packages/beacon-node/src/chain/bls/interface.ts:3-46 and
// packages/state-transition/src/util/signatureSets.ts:5-22.

/** @chainsafe/bls PointFormat */
export declare const PointFormat: {compressed: "compressed"; uncompressed: "uncompressed"};

/**
 * A registered handle, a @chainsafe/bls PublicKey (serialised with toBytes("uncompressed"); a
 * 48-byte result is decompressed on the GPU), or raw 96- / 48-byte encodings.
 */
export type PublicKeyLike = Uint8Array | GpuPublicKey | {toBytes(format?: "compressed" | "uncompressed"): Uint8Array};

export declare const SignatureSetType: {single: "single"; aggregate: "aggregate"};

export type ISignatureSet =
  | {type: "single"; pubkey: PublicKeyLike; signingRoot: Uint8Array; signature: Uint8Array}
  | {type: "aggregate"; pubkeys: PublicKeyLike[]; signingRoot: Uint8Array; signature: Uint8Array};

export type VerifySignatureOpts = {
  batchable?: boolean;
  verifyOnMainThread?: boolean;
};

export interface IBlsVerifier {
  verifySignatureSets(sets: ISignatureSet[], opts?: VerifySignatureOpts): Promise<boolean>;
  close(): Promise<void>;
}

/** beacon-node/src/util/queue/errors.ts:3-6 */
export declare const QueueErrorCode: {
  QUEUE_ABORTED: "QUEUE_ERROR_QUEUE_ABORTED";
  QUEUE_MAX_LENGTH: "QUEUE_ERROR_QUEUE_MAX_LENGTH";
};

/** LodestarError<{code}>: message = type.code */
export declare class QueueError extends Error {
  constructor(type: {code: string});
  type: {code: string};
  getMetadata(): {code: string};
}

/** A key registered in the GPU-resident table (the epoch cache's index2pubkey entry). */
export declare class GpuPublicKey {
  readonly index: number;
  toBytes(): Uint8Array;
}

export declare class BlsGpuVerifier implements IBlsVerifier {
  /** engines: batches in flight on the device (default 2), each with its own streams + workspace; the
   *  pool also creates one engine for verifyOnMainThread calls, so it takes engines + 1 of the
   *  per-device cap (LB_MAX_ENGINES_PER_DEVICE, default 16) */
  /** modules as BlsMultiThreadWorkerPool's: metrics.blsThreadPool.* / metrics.bls.* get the same updates */
  constructor(opts?: {device?: number; engines?: number; blsVerifyAllMultiThread?: boolean},
              modules?: {logger?: {error(msg: string, ctx?: object, e?: Error): void}; metrics?: unknown});
  /** 48- or 96-byte keys -> handles carrying their table index (validate: keyValidate checks) */
  registerPubkeys(keys: Uint8Array[], validate?: boolean): GpuPublicKey[];
  verifySignatureSets(sets: ISignatureSet[], opts?: VerifySignatureOpts): Promise<boolean>;
  /** state-transition verifySignatureSet: synchronous, throws the blst error on malformed input */
  verifySignatureSet(set: ISignatureSet): boolean;
  /** bls.Signature.aggregate(signatures).toBytes() (op pools), 96-byte compressed */
  aggregateSignatures(signatures: Uint8Array[], validate?: boolean): Uint8Array;
  close(): Promise<void>;
  readonly stats: {batches: number; jobs: number; sets: number; batchRetries: number; batchSigsSuccess: number;
    jobsInvalid: number; jobsError: number; jobWaitMs: number; deviceMs: number; mainThreadMs: number};
}

/** light-client isValidBlsAggregate (validation.ts:154-184) with its stage-prefixed errors */
export declare function isValidBlsAggregate(verifier: BlsGpuVerifier, publicKeys: PublicKeyLike[],
                                            message: Uint8Array, signature: Uint8Array): boolean;

export declare function chunkifyMaximizeChunkSize<T>(arr: T[], minPerChunk: number): T[][];
export declare const MAX_SIGNATURE_SETS_PER_JOB: number;
export declare const MAX_BUFFERED_SIGS: number;
export declare const MAX_BUFFER_WAIT_MS: number;
