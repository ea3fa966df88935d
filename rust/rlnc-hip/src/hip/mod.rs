//! `rlnc::full::{Encoder, Decoder, Recoder}` over librlnc_hip (the MI355X engine), behind `--features hip`.
//!
//! Drop-in: same names, signatures, error variants and check order as `src/full/{encoder,decoder,recoder}.rs`;
//! `Clone` + `Debug` like the reference's `#[derive(Clone, Debug)]` (`encoder.rs:18`, `decoder.rs:8`,
//! `recoder.rs:12`); `Send + Sync` like the reference types.  Randomness stays here: the same `rng.fill_bytes`
//! calls as `encoder.rs:248` / `recoder.rs:131` draw the coefficients, and the engine is bit-exact for the same
//! coefficient bytes, so a seeded RNG gives byte-identical pieces on both paths (`tests.rs` checks it).
//! Wired into the crate by `reference.patch` (lib.rs: `mod hip;`, full/mod.rs: the re-export).

mod ffi;
#[cfg(test)]
mod tests;

use crate::RLNCError;
use core::ffi::c_int;
use rand::Rng;
use std::sync::OnceLock;

/// Status code of the C ABI → `Result` (codes 1..=13 are `RLNCError` discriminant + 1, errors.rs:3-32 order).
/// `RLNCError` derives only `Debug, PartialEq` (errors.rs:2), so every variant is built here, not copied.
fn status(s: c_int) -> Result<(), RLNCError> {
    match s {
        ffi::RLNC_OK => Ok(()),
        ffi::RLNC_ERR_CODING_VECTOR_LENGTH_MISMATCH => Err(RLNCError::CodingVectorLengthMismatch),
        ffi::RLNC_ERR_DATA_LENGTH_MISMATCH => Err(RLNCError::DataLengthMismatch),
        ffi::RLNC_ERR_PIECE_COUNT_ZERO => Err(RLNCError::PieceCountZero),
        ffi::RLNC_ERR_DATA_LENGTH_ZERO => Err(RLNCError::DataLengthZero),
        ffi::RLNC_ERR_PIECE_LENGTH_ZERO => Err(RLNCError::PieceLengthZero),
        ffi::RLNC_ERR_NOT_ENOUGH_PIECES_TO_RECODE => Err(RLNCError::NotEnoughPiecesToRecode),
        ffi::RLNC_ERR_PIECE_LENGTH_TOO_SHORT => Err(RLNCError::PieceLengthTooShort),
        ffi::RLNC_ERR_PIECE_NOT_USEFUL => Err(RLNCError::PieceNotUseful),
        ffi::RLNC_ERR_RECEIVED_ALL_PIECES => Err(RLNCError::ReceivedAllPieces),
        ffi::RLNC_ERR_NOT_ALL_PIECES_RECEIVED_YET => Err(RLNCError::NotAllPiecesReceivedYet),
        ffi::RLNC_ERR_INVALID_DECODED_DATA_FORMAT => Err(RLNCError::InvalidDecodedDataFormat),
        ffi::RLNC_ERR_INVALID_PIECE_LENGTH => Err(RLNCError::InvalidPieceLength),
        ffi::RLNC_ERR_INVALID_OUTPUT_BUFFER => Err(RLNCError::InvalidOutputBuffer),
        // No reference variant (device fault, allocation failure, misuse of the ABI): fail loudly, never fall
        // back to the CPU path.
        _ => engine_failure(s),
    }
}

#[cold]
fn engine_failure(s: c_int) -> ! {
    // SAFETY: rlnc_last_error returns a NUL-terminated thread-local string owned by the library.
    let msg = unsafe { std::ffi::CStr::from_ptr(ffi::rlnc_last_error()) };
    panic!("librlnc_hip engine error {s}: {}", msg.to_string_lossy())
}

/// One process-wide context on device `RLNC_HIP_DEVICE` (default 0).  The object API is thread-safe on one
/// context (every call leases its own stream and buffers) and each object holds its own reference on it
/// (include/rlnc_hip.h, "Threading" / "Lifetime"), so it is never destroyed.
struct Ctx(*mut ffi::rlnc_context);
// SAFETY: the context is internally synchronised (include/rlnc_hip.h, "Threading").
unsafe impl Send for Ctx {}
unsafe impl Sync for Ctx {}

fn ctx() -> *mut ffi::rlnc_context {
    static CTX: OnceLock<Ctx> = OnceLock::new();
    CTX.get_or_init(|| {
        let device = std::env::var("RLNC_HIP_DEVICE").ok().and_then(|v| v.parse().ok()).unwrap_or(0);
        let mut c = core::ptr::null_mut();
        // SAFETY: out-pointer to a local.
        let s = unsafe { ffi::rlnc_context_create(device, &mut c) };
        if s != ffi::RLNC_OK {
            engine_failure(s);
        }
        Ctx(c)
    })
    .0
}

macro_rules! handle {
    ($T:ident, $raw:ty, $clone:path, $free:path) => {
        pub struct $T {
            h: *mut $raw,
        }
        // SAFETY: Encoder::code_with_buf(&self) is safe from many threads on one handle (per-call streams and
        // workspaces); the &self methods of Decoder / Recoder only read, and &mut self gives exclusive access.
        unsafe impl Send for $T {}
        unsafe impl Sync for $T {}
        impl Clone for $T {
            // #[derive(Clone)] of the reference types: an independent deep copy (device state included)
            fn clone(&self) -> Self {
                let mut h = core::ptr::null_mut();
                // SAFETY: self.h is a live handle; out-pointer to a local.
                let s = unsafe { $clone(self.h, &mut h) };
                if s != ffi::RLNC_OK {
                    engine_failure(s);
                }
                $T { h }
            }
        }
        impl Drop for $T {
            fn drop(&mut self) {
                // SAFETY: the handle is owned and freed exactly once.
                unsafe { $free(self.h) }
            }
        }
    };
}
handle!(Encoder, ffi::rlnc_encoder, ffi::rlnc_encoder_clone, ffi::rlnc_encoder_free);
handle!(Decoder, ffi::rlnc_decoder, ffi::rlnc_decoder_clone, ffi::rlnc_decoder_free);
handle!(Recoder, ffi::rlnc_recoder, ffi::rlnc_recoder_clone, ffi::rlnc_recoder_free);

impl Encoder {
    /// encoder.rs:27-29
    pub fn get_piece_count(&self) -> usize {
        unsafe { ffi::rlnc_encoder_get_piece_count(self.h) }
    }
    /// encoder.rs:32-34
    pub fn get_piece_byte_len(&self) -> usize {
        unsafe { ffi::rlnc_encoder_get_piece_byte_len(self.h) }
    }
    /// encoder.rs:37-39
    pub fn get_full_coded_piece_byte_len(&self) -> usize {
        unsafe { ffi::rlnc_encoder_get_full_coded_piece_byte_len(self.h) }
    }

    /// encoder.rs:50-71 (crate-private, as in the reference)
    #[allow(dead_code)]
    pub(crate) fn without_padding(data: Vec<u8>, piece_count: usize) -> Result<Encoder, RLNCError> {
        let mut h = core::ptr::null_mut();
        status(unsafe { ffi::rlnc_encoder_without_padding(ctx(), data.as_ptr(), data.len(), piece_count, &mut h) })?;
        Ok(Encoder { h })
    }

    /// encoder.rs:85-106: pads with the 0x81 marker and zeros, splits into `piece_count` pieces.
    pub fn new(data: Vec<u8>, piece_count: usize) -> Result<Encoder, RLNCError> {
        let mut h = core::ptr::null_mut();
        status(unsafe { ffi::rlnc_encoder_new(ctx(), data.as_ptr(), data.len(), piece_count, &mut h) })?;
        Ok(Encoder { h })
    }

    /// encoder.rs:128-144 (crate-private, as in the reference): coded_data = Σ coding_vector[i] · piece_i.
    #[allow(dead_code)]
    pub(crate) fn code_with_coding_vector(&self, coding_vector: &[u8], coded_data: &mut [u8]) -> Result<(), RLNCError> {
        status(unsafe {
            ffi::rlnc_encoder_code_with_coding_vector(
                self.h,
                coding_vector.as_ptr(),
                coding_vector.len(),
                coded_data.as_mut_ptr(),
                coded_data.len(),
            )
        })
    }

    /// encoder.rs:241-250: length check first (InvalidOutputBuffer), then `rng.fill_bytes` into the coefficient
    /// prefix, then the data part.
    pub fn code_with_buf<R: Rng + ?Sized>(&self, rng: &mut R, full_coded_piece: &mut [u8]) -> Result<(), RLNCError> {
        if full_coded_piece.len() != self.get_full_coded_piece_byte_len() {
            return Err(RLNCError::InvalidOutputBuffer);
        }
        let k = self.get_piece_count();
        rng.fill_bytes(&mut full_coded_piece[..k]);
        // The engine reads the k coefficient bytes before it writes coeffs ‖ data into the same buffer; both
        // pointers come from one raw pointer.
        let p = full_coded_piece.as_mut_ptr();
        status(unsafe { ffi::rlnc_encoder_code_with_buf(self.h, p as *const u8, k, p, full_coded_piece.len()) })
    }

    /// encoder.rs:264-269
    pub fn code<R: Rng + ?Sized>(&self, rng: &mut R) -> Vec<u8> {
        let mut full_coded_piece = vec![0u8; self.get_full_coded_piece_byte_len()];
        match self.code_with_buf(rng, &mut full_coded_piece) {
            Ok(()) => full_coded_piece,
            Err(e) => unreachable!("the output buffer has the exact length: {e:?}"),
        }
    }
}

impl Decoder {
    /// decoder.rs:25-27
    pub fn get_num_pieces_coded_together(&self) -> usize {
        unsafe { ffi::rlnc_decoder_get_num_pieces_coded_together(self.h) }
    }
    /// decoder.rs:30-32
    pub fn get_piece_byte_len(&self) -> usize {
        unsafe { ffi::rlnc_decoder_get_piece_byte_len(self.h) }
    }
    /// decoder.rs:35-37
    pub fn get_full_coded_piece_byte_len(&self) -> usize {
        unsafe { ffi::rlnc_decoder_get_full_coded_piece_byte_len(self.h) }
    }
    /// decoder.rs:40-42
    pub fn get_received_piece_count(&self) -> usize {
        unsafe { ffi::rlnc_decoder_get_received_piece_count(self.h) }
    }
    /// decoder.rs:45-47
    pub fn get_useful_piece_count(&self) -> usize {
        unsafe { ffi::rlnc_decoder_get_useful_piece_count(self.h) }
    }
    /// decoder.rs:50-52
    pub fn get_remaining_piece_count(&self) -> usize {
        unsafe { ffi::rlnc_decoder_get_remaining_piece_count(self.h) }
    }

    /// decoder.rs:65-80 (argument order: piece length first, then the piece count).
    pub fn new(piece_byte_len: usize, required_piece_count: usize) -> Result<Decoder, RLNCError> {
        let mut h = core::ptr::null_mut();
        status(unsafe { ffi::rlnc_decoder_new(ctx(), piece_byte_len, required_piece_count, &mut h) })?;
        Ok(Decoder { h })
    }

    /// decoder.rs:96-118: Ok / PieceNotUseful / ReceivedAllPieces / InvalidPieceLength, answered immediately
    /// (the exact diagonal-pivot elimination of the coefficient block); invalid input leaves the state unchanged.
    pub fn decode(&mut self, full_coded_piece: &[u8]) -> Result<(), RLNCError> {
        status(unsafe { ffi::rlnc_decoder_decode(self.h, full_coded_piece.as_ptr(), full_coded_piece.len()) })
    }

    /// decoder.rs:121-123
    pub fn is_already_decoded(&self) -> bool {
        unsafe { ffi::rlnc_decoder_is_already_decoded(self.h) != 0 }
    }

    /// decoder.rs:136-159: consumes the decoder, like the reference.
    pub fn get_decoded_data(self) -> Result<Vec<u8>, RLNCError> {
        let mut out = vec![0u8; self.get_num_pieces_coded_together() * self.get_piece_byte_len()];
        let mut len = 0usize;
        status(unsafe { ffi::rlnc_decoder_get_decoded_data(self.h, out.as_mut_ptr(), out.len(), &mut len) })?;
        out.truncate(len);
        Ok(out)
    }
}

impl Recoder {
    /// recoder.rs:26-28
    pub fn get_original_num_pieces_coded_together(&self) -> usize {
        unsafe { ffi::rlnc_recoder_get_original_num_pieces_coded_together(self.h) }
    }
    /// recoder.rs:31-33
    pub fn get_num_pieces_recoded_together(&self) -> usize {
        unsafe { ffi::rlnc_recoder_get_num_pieces_recoded_together(self.h) }
    }
    /// recoder.rs:36-38
    pub fn get_piece_byte_len(&self) -> usize {
        unsafe { ffi::rlnc_recoder_get_piece_byte_len(self.h) }
    }
    /// recoder.rs:41-43
    pub fn get_full_coded_piece_byte_len(&self) -> usize {
        unsafe { ffi::rlnc_recoder_get_full_coded_piece_byte_len(self.h) }
    }

    /// recoder.rs:68-108; same check order (NotEnoughPiecesToRecode, PieceLengthZero, PieceCountZero,
    /// PieceLengthTooShort).  `0 < data.len() < full_coded_piece_byte_len` is undefined behaviour in the reference
    /// (`unwrap_unchecked` on an `Err`, recoder.rs:97); here it is `Err(NotEnoughPiecesToRecode)`.
    pub fn new(data: Vec<u8>, full_coded_piece_byte_len: usize, num_pieces_coded_together: usize) -> Result<Recoder, RLNCError> {
        let mut h = core::ptr::null_mut();
        status(unsafe {
            ffi::rlnc_recoder_new(
                ctx(),
                data.as_ptr(),
                data.len(),
                full_coded_piece_byte_len,
                num_pieces_coded_together,
                &mut h,
            )
        })?;
        Ok(Recoder { h })
    }

    /// recoder.rs:122-153: length check first, then `rng.fill_bytes` of the n recoding coefficients.
    pub fn recode_with_buf<R: Rng + ?Sized>(&mut self, rng: &mut R, full_recoded_piece: &mut [u8]) -> Result<(), RLNCError> {
        if full_recoded_piece.len() != self.get_full_coded_piece_byte_len() {
            return Err(RLNCError::InvalidOutputBuffer);
        }
        let mut r = vec![0u8; self.get_num_pieces_recoded_together()];
        rng.fill_bytes(&mut r);
        status(unsafe {
            ffi::rlnc_recoder_recode_with_buf(
                self.h,
                r.as_ptr(),
                r.len(),
                full_recoded_piece.as_mut_ptr(),
                full_recoded_piece.len(),
            )
        })
    }

    /// recoder.rs:166-171
    pub fn recode<R: Rng + ?Sized>(&mut self, rng: &mut R) -> Vec<u8> {
        let mut full_recoded_piece = vec![0u8; self.get_full_coded_piece_byte_len()];
        match self.recode_with_buf(rng, &mut full_recoded_piece) {
            Ok(()) => full_recoded_piece,
            Err(e) => unreachable!("the output buffer has the exact length: {e:?}"),
        }
    }
}

impl core::fmt::Debug for Encoder {
    fn fmt(&self, f: &mut core::fmt::Formatter<'_>) -> core::fmt::Result {
        f.debug_struct("Encoder")
            .field("piece_count", &self.get_piece_count())
            .field("piece_byte_len", &self.get_piece_byte_len())
            .finish_non_exhaustive()
    }
}

impl core::fmt::Debug for Decoder {
    fn fmt(&self, f: &mut core::fmt::Formatter<'_>) -> core::fmt::Result {
        f.debug_struct("Decoder")
            .field("required_piece_count", &self.get_num_pieces_coded_together())
            .field("piece_byte_len", &self.get_piece_byte_len())
            .field("received_piece_count", &self.get_received_piece_count())
            .field("useful_piece_count", &self.get_useful_piece_count())
            .finish_non_exhaustive()
    }
}

impl core::fmt::Debug for Recoder {
    fn fmt(&self, f: &mut core::fmt::Formatter<'_>) -> core::fmt::Result {
        f.debug_struct("Recoder")
            .field("num_pieces_received", &self.get_num_pieces_recoded_together())
            .field("full_coded_piece_byte_len", &self.get_full_coded_piece_byte_len())
            .finish_non_exhaustive()
    }
}
