// Type declarations for the MI355X IBlsVerifier drop-in (lodestar_amd/js/index.js).
// Mirrors packages/beacon-node/src/chain/bls/interface.ts:3-46 and
// packages/state-transition/src/util/signatureSets.ts:5-22.

export type PublicKeyLike = Uint8Array | GpuPublicKey | {toBytes(): Uint8Array};

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

export declare class QueueError extends Error {
  type: {code: string};
}

/** A key registered in the GPU-resident table (the epoch cache's index2pubkey entry). */
export declare class GpuPublicKey {
  readonly index: number;
  toBytes(): Uint8Array;
}

export declare class BlsGpuVerifier implements IBlsVerifier {
  /** engines: batches in flight on the device (default 2), each with its own streams + workspace */
  constructor(opts?: {device?: number; engines?: number; blsVerifyAllMultiThread?: boolean});
  /** 48- or 96-byte keys -> handles carrying their table index (validate: keyValidate checks) */
  registerPubkeys(keys: Uint8Array[], validate?: boolean): GpuPublicKey[];
  verifySignatureSets(sets: ISignatureSet[], opts?: VerifySignatureOpts): Promise<boolean>;
  /** state-transition verifySignatureSet: synchronous, throws the blst error on malformed input */
  verifySignatureSet(set: ISignatureSet): boolean;
  /** bls.Signature.aggregate(signatures).toBytes() (op pools), 96-byte compressed */
  aggregateSignatures(signatures: Uint8Array[], validate?: boolean): Uint8Array;
  close(): Promise<void>;
  readonly stats: {batches: number; jobs: number; sets: number; jobsInvalid: number; jobsError: number};
}

/** light-client isValidBlsAggregate (validation.ts:154-184) with its stage-prefixed errors */
export declare function isValidBlsAggregate(verifier: BlsGpuVerifier, publicKeys: PublicKeyLike[],
                                            message: Uint8Array, signature: Uint8Array): boolean;

export declare function chunkifyMaximizeChunkSize<T>(arr: T[], minPerChunk: number): T[][];
export declare const MAX_SIGNATURE_SETS_PER_JOB: number;
export declare const MAX_BUFFERED_SIGS: number;
export declare const MAX_BUFFER_WAIT_MS: number;
