//! mysticeti-core/src/gpu_verify.rs (new file): StatementBlock::verify on the MI355X engine.
//!
//! One `mv_verify_blocks` call checks a whole message worth of blocks on the GPU (bincode
//! parse, both BLAKE2b-256 digests, the ZIP-215 signature and every structural check, in the
//! order of types.rs:315-376). The engine returns one status per block; this wrapper turns a
//! failing status back into the exact `eyre` error `StatementBlock::verify` would have
//! returned. The message text needs the failing values (digests, the include, the range), so
//! for a rejected block the wrapper re-reads them host-side -- only on that failure path.
use std::sync::Arc;

use eyre::{bail, ensure};
use mysti_verify_sys as sys;

use crate::committee::Committee;
use crate::crypto::BlockDigest;
use crate::data::Data;
use crate::serde::ByteRepr; // serde.rs:8-14
use crate::types::{BaseStatement, StatementBlock};

pub struct GpuVerifier {
    ctx: *mut sys::mv_ctx,
}
// mv_* calls are thread-safe on one context; concurrent callers are merged by the engine's
// submission queue (one device pass serves all of them)
unsafe impl Send for GpuVerifier {}
unsafe impl Sync for GpuVerifier {}

impl Drop for GpuVerifier {
    fn drop(&mut self) {
        unsafe { sys::mv_destroy(self.ctx) }
    }
}

impl GpuVerifier {
    /// Opens the devices in `device_mask` and loads the committee (keys decoded once per
    /// device, as Committee::load decodes each VerificationKey once, committee.rs:83-87).
    pub fn new(committee: &Committee, device_mask: u32) -> eyre::Result<Arc<Self>> {
        let mut ctx = std::ptr::null_mut();
        let cfg = sys::mv_config { device_mask, ..Default::default() };
        ensure!(unsafe { sys::mv_create(&cfg, &mut ctx) } == sys::MV_OK, "no gfx950 device in mask {device_mask:#x}");
        let me = Self { ctx };
        let pks: Vec<u8> = committee
            .authorities()
            .flat_map(|a| committee.get_public_key(a).unwrap().0.as_bytes().to_vec())
            .collect();
        let stakes: Vec<u64> = committee.authorities().map(|a| committee.get_stake(a).unwrap()).collect();
        let rc = unsafe {
            sys::mv_set_committee(me.ctx, pks.as_ptr(), stakes.as_ptr(), stakes.len() as u32, committee.epoch(),
                                  std::ptr::null_mut())
        };
        ensure!(rc == sys::MV_OK, "mv_set_committee: {}", me.last_error());
        Ok(Arc::new(me))
    }

    fn last_error(&self) -> String {
        unsafe { std::ffi::CStr::from_ptr(sys::mv_last_error(self.ctx)) }.to_string_lossy().into_owned()
    }

    /// StatementBlock::verify (types.rs:315-376) for every block, same results, same errors.
    pub fn verify_blocks(&self, blocks: &[Data<StatementBlock>], committee: &Committee) -> Vec<eyre::Result<()>> {
        let mut buf = Vec::new();
        let mut off = Vec::with_capacity(blocks.len());
        let mut len = Vec::with_capacity(blocks.len());
        for b in blocks {
            off.push(buf.len() as u64);
            len.push(b.serialized_bytes().len() as u64);
            buf.extend_from_slice(b.serialized_bytes());
        }
        let mut status = vec![0u8; blocks.len()];
        let mut digest = vec![0u8; 32 * blocks.len()];
        let rc = unsafe {
            sys::mv_verify_blocks(self.ctx, buf.as_ptr(), off.as_ptr(), len.as_ptr(), blocks.len() as u32,
                                  status.as_mut_ptr(), std::ptr::null_mut(), digest.as_mut_ptr())
        };
        if rc != sys::MV_OK {
            let e = self.last_error();
            return blocks.iter().map(|_| Err(eyre::eyre!("GPU verifier failed: {e}"))).collect();
        }
        blocks
            .iter()
            .zip(status)
            .zip(digest.chunks(32))
            .map(|((b, s), d)| verdict_to_result(b, s, d, committee))
            .collect()
    }
}

/// The blocks of received network frames (network.rs:400-447: u32 BE size + bincode
/// NetworkMessage) as (offsets, lengths) into `buf`, and the bytes of the complete frames: a
/// receiver that reads frames into one buffer passes it and these arrays to mv_verify_blocks
/// without deserializing. An error where Network::handle_read_stream drops the connection.
pub fn frame_blocks(buf: &[u8]) -> eyre::Result<(Vec<u64>, Vec<u64>, usize)> {
    let mut consumed = 0u64;
    let n = unsafe {
        sys::mv_frame_blocks(buf.as_ptr(), buf.len() as u64, std::ptr::null_mut(), std::ptr::null_mut(), 0,
                             &mut consumed)
    };
    ensure!(n >= 0, "malformed frame stream");
    let mut off = vec![0u64; n as usize];
    let mut len = vec![0u64; n as usize];
    unsafe {
        sys::mv_frame_blocks(buf.as_ptr(), buf.len() as u64, off.as_mut_ptr(), len.as_mut_ptr(), n as u64,
                             &mut consumed)
    };
    Ok((off, len, consumed as usize))
}

/// The error StatementBlock::verify returns for the check the engine reports as failing.
fn verdict_to_result(block: &StatementBlock, status: u8, digest: &[u8], committee: &Committee) -> eyre::Result<()> {
    let round = block.round();
    match status {
        sys::MV_BLOCK_OK => Ok(()),
        // types.rs:327-332
        sys::MV_BLOCK_DIGEST_MISMATCH => bail!(
            "Digest does not match, calculated {:?}, provided {:?}",
            <BlockDigest as ByteRepr>::try_copy_from_slice::<serde::de::value::Error>(digest).unwrap(),
            block.digest()
        ),
        // types.rs:333-338
        sys::MV_BLOCK_EPOCH_MISMATCH => bail!(
            "Block's epoch {} doesn't match committee epoch {}",
            block.epoch(),
            committee.epoch()
        ),
        // types.rs:339-342
        sys::MV_BLOCK_UNKNOWN_AUTHOR => bail!("Unknown block author {}", block.author()),
        // types.rs:343-345
        sys::MV_BLOCK_GENESIS => bail!("Genesis block should not go through verification"),
        // types.rs:346-348 (committee keys decode at Committee::load, so the error is InvalidSignature)
        sys::MV_BLOCK_SIG_INVALID => bail!(
            "Block signature verification has failed: {:?}",
            ed25519_consensus::Error::InvalidSignature
        ),
        // types.rs:349-362: the first failing include, checked in the reference's order
        sys::MV_BLOCK_INCLUDE_UNKNOWN_AUTHORITY | sys::MV_BLOCK_INCLUDE_ROUND => {
            for include in block.includes() {
                ensure!(
                    committee.known_authority(include.authority),
                    "Include {:?} references unknown authority",
                    include
                );
                ensure!(
                    include.round < round,
                    "Include {:?} round is greater or equal to own round {}",
                    include,
                    round
                );
            }
            unreachable!("engine reported a failing include")
        }
        // types.rs:363-370 -> VoteRange::verify (types.rs:440-460): its own error, first failing range
        sys::MV_BLOCK_VOTE_RANGE | sys::MV_BLOCK_VOTE_RANGE_TOO_LONG | sys::MV_BLOCK_VOTE_RANGE_END_TOO_LARGE => {
            for statement in block.statements() {
                if let BaseStatement::VoteRange(range) = statement {
                    range.verify()?;
                }
            }
            unreachable!("engine reported a failing VoteRange")
        }
        // types.rs:371-374
        sys::MV_BLOCK_THRESHOLD_CLOCK => bail!("Threshold clock is not valid"),
        // bincode::deserialize failed (Data::from_bytes, data.rs:43-52, happens before verify in
        // the reference); blocks arriving here were already deserialized, so this is unreachable
        _ => bail!("block bytes do not deserialize"),
    }
}
