// Type declarations for the MI355X IBlsVerifier drop-in (lodestar_amd/js/index.js).
// Mirrors packages/beacon-node/src/chain/bls/interface.ts:3-46 and
// packages/state-transition/src/util/signatureSets.ts:5-22.

export type PublicKeyLike = Uint8Array | {toBytes(): Uint8Array};

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

export declare class BlsGpuVerifier implements IBlsVerifier {
  constructor(opts?: {device?: number; blsVerifyAllMultiThread?: boolean});
  verifySignatureSets(sets: ISignatureSet[], opts?: VerifySignatureOpts): Promise<boolean>;
  close(): Promise<void>;
}

export declare function chunkifyMaximizeChunkSize<T>(arr: T[], minPerChunk: number): T[][];
export declare const MAX_SIGNATURE_SETS_PER_JOB: number;
export declare const MAX_BUFFERED_SIGS: number;
export declare const MAX_BUFFER_WAIT_MS: number;
