//! Raw declarations of `include/rlnc_hip.h` (librlnc_hip.so, the MI355X engine for rlnc's hot path).
//!
//! Every function and struct of the header is declared here with the same name, argument order and C types
//! (`size_t` = `usize`, `int` = `c_int`, `uint8_t *` = `*mut u8`, ...).  `tests/test_rust_shim.py` in the
//! librlnc_hip repository parses this file and the header and fails on any difference, so the two cannot drift.
//! Edition 2024 (the crate's `Cargo.toml:4`): foreign blocks are `unsafe extern`.
#![allow(non_camel_case_types, non_snake_case, dead_code)]

use core::ffi::{c_char, c_int, c_void};

// ---- status codes: RLNCError discriminant + 1 (src/common/errors.rs:3-32), engine errors >= 100 ----
pub const RLNC_OK: c_int = 0;
pub const RLNC_ERR_CODING_VECTOR_LENGTH_MISMATCH: c_int = 1;
pub const RLNC_ERR_DATA_LENGTH_MISMATCH: c_int = 2;
pub const RLNC_ERR_PIECE_COUNT_ZERO: c_int = 3;
pub const RLNC_ERR_DATA_LENGTH_ZERO: c_int = 4;
pub const RLNC_ERR_PIECE_LENGTH_ZERO: c_int = 5;
pub const RLNC_ERR_NOT_ENOUGH_PIECES_TO_RECODE: c_int = 6;
pub const RLNC_ERR_PIECE_LENGTH_TOO_SHORT: c_int = 7;
pub const RLNC_ERR_PIECE_NOT_USEFUL: c_int = 8;
pub const RLNC_ERR_RECEIVED_ALL_PIECES: c_int = 9;
pub const RLNC_ERR_NOT_ALL_PIECES_RECEIVED_YET: c_int = 10;
pub const RLNC_ERR_INVALID_DECODED_DATA_FORMAT: c_int = 11;
pub const RLNC_ERR_INVALID_PIECE_LENGTH: c_int = 12;
pub const RLNC_ERR_INVALID_OUTPUT_BUFFER: c_int = 13;
pub const RLNC_ERR_INVALID_ARGUMENT: c_int = 100;
pub const RLNC_ERR_DEVICE: c_int = 101;
pub const RLNC_ERR_OUT_OF_MEMORY: c_int = 102;
pub const RLNC_ERR_NO_DEVICE: c_int = 103;

// ---- opaque handles ----
#[repr(C)]
pub struct rlnc_context {
    _p: [u8; 0],
}
#[repr(C)]
pub struct rlnc_encoder {
    _p: [u8; 0],
}
#[repr(C)]
pub struct rlnc_decoder {
    _p: [u8; 0],
}
#[repr(C)]
pub struct rlnc_recoder {
    _p: [u8; 0],
}
#[repr(C)]
pub struct rlnc_elimination {
    _p: [u8; 0],
}

// ---- descriptors (field order and types as in the header) ----
#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct rlnc_matmul_desc {
    pub in_: *const u8,
    pub in_obj_stride: i64,
    pub in_row_stride: i64,
    pub coef: *const u8,
    pub coef_obj_stride: i64,
    pub coef_row_stride: i64,
    pub out: *mut u8,
    pub out_obj_stride: i64,
    pub out_row_stride: i64,
    pub hdr: *mut u8,
    pub hdr_obj_stride: i64,
    pub hdr_row_stride: i64,
    pub n_out: i32,
    pub n_in: i32,
    pub width: i64,
    pub n_obj: i32,
}

#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct rlnc_pad_desc {
    pub data: *const u8,
    pub data_len: usize,
    pub k: usize,
    pub out: *mut u8,
    pub out_row_stride: usize,
}

#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct rlnc_object_desc {
    pub src: *const u8,
    pub src_row_stride: usize,
    pub coeffs: *const u8,
    pub pieces: *mut u8,
    pub piece_row_stride: usize,
    pub k: usize,
    pub L: usize,
    pub n: usize,
}

#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct rlnc_recode_object_desc {
    pub pieces: *const u8,
    pub piece_row_stride: usize,
    pub r: *const u8,
    pub out: *mut u8,
    pub out_row_stride: usize,
    pub k: usize,
    pub L: usize,
    pub n: usize,
    pub n_recoded: usize,
}

#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct rlnc_decode_object_desc {
    pub pieces: *const u8,
    pub piece_row_stride: usize,
    pub decoded: *mut u8,
    pub k: usize,
    pub L: usize,
    pub m: usize,
}

unsafe extern "C" {
    // status text, errors.rs:34-58
    pub fn rlnc_status_name(status: c_int) -> *const c_char;
    pub fn rlnc_status_message(status: c_int) -> *const c_char;
    pub fn rlnc_last_error() -> *const c_char;
    pub fn rlnc_version() -> *const c_char;

    // context
    pub fn rlnc_context_create(device: c_int, out: *mut *mut rlnc_context) -> c_int;
    pub fn rlnc_context_destroy(ctx: *mut rlnc_context);
    pub fn rlnc_context_set_stream(ctx: *mut rlnc_context, hip_stream: *mut c_void) -> c_int;
    pub fn rlnc_context_use_own_stream(ctx: *mut rlnc_context) -> c_int;
    pub fn rlnc_context_get_stream(ctx: *mut rlnc_context) -> *mut c_void;
    pub fn rlnc_context_synchronize(ctx: *mut rlnc_context) -> c_int;
    pub fn rlnc_context_device(ctx: *const rlnc_context) -> c_int;
    pub fn rlnc_stream_is_capturing(hip_stream: *mut c_void, capturing: *mut c_int) -> c_int;
    pub fn rlnc_device_unaligned_vector_access(device: c_int) -> c_int;

    // L1 vector primitives, src/common/simd/mod.rs:18-119 (device buffers)
    pub fn rlnc_gf256_inplace_mul_vec_by_scalar(ctx: *mut rlnc_context, vec_dev: *mut u8, len: usize, scalar: u8)
    -> c_int;
    pub fn rlnc_gf256_inplace_add_vectors(ctx: *mut rlnc_context, dst_dev: *mut u8, src_dev: *const u8, len: usize)
    -> c_int;
    pub fn rlnc_gf256_mul_vec_by_scalar_then_add_into_vec(
        ctx: *mut rlnc_context,
        dst_dev: *mut u8,
        src_dev: *const u8,
        len: usize,
        scalar: u8,
    ) -> c_int;

    // L2 matrix operator
    pub fn rlnc_gf256_matmul(ctx: *mut rlnc_context, desc: *const rlnc_matmul_desc) -> c_int;
    pub fn rlnc_set_kernel_variant(ctx: *mut rlnc_context, variant: c_int, max_tile_rows: c_int) -> c_int;
    pub fn rlnc_set_column_run(ctx: *mut rlnc_context, col_run: c_int) -> c_int;
    pub fn rlnc_set_decode_path(ctx: *mut rlnc_context, path: c_int) -> c_int;

    // Encoder: encoder.rs:18 (Clone), :27-39, :50-71, :85-106, :128-144, :241-250
    pub fn rlnc_encoder_new(
        ctx: *mut rlnc_context,
        data: *const u8,
        data_len: usize,
        piece_count: usize,
        out: *mut *mut rlnc_encoder,
    ) -> c_int;
    pub fn rlnc_encoder_without_padding(
        ctx: *mut rlnc_context,
        data: *const u8,
        data_len: usize,
        piece_count: usize,
        out: *mut *mut rlnc_encoder,
    ) -> c_int;
    pub fn rlnc_encoder_from_device(
        ctx: *mut rlnc_context,
        pieces_dev: *const u8,
        piece_count: usize,
        piece_len: usize,
        row_stride: usize,
        out: *mut *mut rlnc_encoder,
    ) -> c_int;
    pub fn rlnc_encoder_clone(enc: *const rlnc_encoder, out: *mut *mut rlnc_encoder) -> c_int;
    pub fn rlnc_encoder_free(enc: *mut rlnc_encoder);
    pub fn rlnc_encoder_get_piece_count(enc: *const rlnc_encoder) -> usize;
    pub fn rlnc_encoder_get_piece_byte_len(enc: *const rlnc_encoder) -> usize;
    pub fn rlnc_encoder_get_full_coded_piece_byte_len(enc: *const rlnc_encoder) -> usize;
    pub fn rlnc_encoder_code_with_coding_vector(
        enc: *mut rlnc_encoder,
        coding_vector: *const u8,
        cv_len: usize,
        coded_data: *mut u8,
        coded_len: usize,
    ) -> c_int;
    pub fn rlnc_encoder_code_with_buf(
        enc: *mut rlnc_encoder,
        random_bytes: *const u8,
        n_random: usize,
        full_coded_piece: *mut u8,
        full_len: usize,
    ) -> c_int;
    pub fn rlnc_encoder_code_batch_device(
        enc: *mut rlnc_encoder,
        coeffs_dev: *const u8,
        n: usize,
        out_dev: *mut u8,
        out_row_stride: usize,
    ) -> c_int;

    // Recoder: recoder.rs:12 (Clone), :26-43, :68-108, :122-171
    pub fn rlnc_recoder_new(
        ctx: *mut rlnc_context,
        data: *const u8,
        data_len: usize,
        full_coded_piece_byte_len: usize,
        num_pieces_coded_together: usize,
        out: *mut *mut rlnc_recoder,
    ) -> c_int;
    pub fn rlnc_recoder_clone(rec: *const rlnc_recoder, out: *mut *mut rlnc_recoder) -> c_int;
    pub fn rlnc_recoder_free(rec: *mut rlnc_recoder);
    pub fn rlnc_recoder_get_original_num_pieces_coded_together(rec: *const rlnc_recoder) -> usize;
    pub fn rlnc_recoder_get_num_pieces_recoded_together(rec: *const rlnc_recoder) -> usize;
    pub fn rlnc_recoder_get_piece_byte_len(rec: *const rlnc_recoder) -> usize;
    pub fn rlnc_recoder_get_full_coded_piece_byte_len(rec: *const rlnc_recoder) -> usize;
    pub fn rlnc_recoder_recode_with_buf(
        rec: *mut rlnc_recoder,
        random_bytes: *const u8,
        n_random: usize,
        full_recoded_piece: *mut u8,
        full_len: usize,
    ) -> c_int;
    pub fn rlnc_recoder_recode_batch_device(
        rec: *mut rlnc_recoder,
        r_dev: *const u8,
        count: usize,
        out_dev: *mut u8,
    ) -> c_int;

    // Decoder: decoder.rs:8 (Clone), :25-52, :65-80, :96-123, :136-177
    pub fn rlnc_decoder_new(
        ctx: *mut rlnc_context,
        piece_byte_len: usize,
        required_piece_count: usize,
        out: *mut *mut rlnc_decoder,
    ) -> c_int;
    pub fn rlnc_decoder_clone(dec: *const rlnc_decoder, out: *mut *mut rlnc_decoder) -> c_int;
    pub fn rlnc_decoder_free(dec: *mut rlnc_decoder);
    pub fn rlnc_decoder_decode(dec: *mut rlnc_decoder, full_coded_piece: *const u8, len: usize) -> c_int;
    pub fn rlnc_decoder_decode_device(dec: *mut rlnc_decoder, piece_dev: *const u8, len: usize) -> c_int;
    pub fn rlnc_decoder_is_already_decoded(dec: *const rlnc_decoder) -> c_int;
    pub fn rlnc_decoder_get_num_pieces_coded_together(dec: *const rlnc_decoder) -> usize;
    pub fn rlnc_decoder_get_piece_byte_len(dec: *const rlnc_decoder) -> usize;
    pub fn rlnc_decoder_get_full_coded_piece_byte_len(dec: *const rlnc_decoder) -> usize;
    pub fn rlnc_decoder_get_received_piece_count(dec: *const rlnc_decoder) -> usize;
    pub fn rlnc_decoder_get_useful_piece_count(dec: *const rlnc_decoder) -> usize;
    pub fn rlnc_decoder_get_remaining_piece_count(dec: *const rlnc_decoder) -> usize;
    pub fn rlnc_decoder_get_decoded_data(dec: *mut rlnc_decoder, out: *mut u8, out_cap: usize, out_len: *mut usize)
    -> c_int;
    pub fn rlnc_decoder_get_decoded_data_device(
        dec: *mut rlnc_decoder,
        out_dev: *mut u8,
        out_cap: usize,
        out_len: *mut usize,
    ) -> c_int;

    // multi-object batch API (device-resident)
    pub fn rlnc_encode_batch(
        ctx: *mut rlnc_context,
        src_dev: *const u8,
        k: usize,
        L: usize,
        num_objects: usize,
        coeffs_dev: *const u8,
        n: usize,
        pieces_dev: *mut u8,
    ) -> c_int;
    pub fn rlnc_encode_batch_headers(
        ctx: *mut rlnc_context,
        coeffs_dev: *const u8,
        k: usize,
        L: usize,
        num_objects: usize,
        n: usize,
        pieces_dev: *mut u8,
    ) -> c_int;
    pub fn rlnc_encode_batch_data(
        ctx: *mut rlnc_context,
        src_dev: *const u8,
        k: usize,
        L: usize,
        num_objects: usize,
        coeffs_dev: *const u8,
        n: usize,
        pieces_dev: *mut u8,
    ) -> c_int;
    pub fn rlnc_encode_batch_plan_bytes(k: usize, num_objects: usize, n: usize) -> usize;
    pub fn rlnc_encode_batch_prepare(
        ctx: *mut rlnc_context,
        src_dev: *const u8,
        k: usize,
        L: usize,
        num_objects: usize,
        coeffs_dev: *const u8,
        n: usize,
        pieces_dev: *mut u8,
        plan_dev: *mut c_void,
        plan_bytes: usize,
    ) -> c_int;
    pub fn rlnc_encode_batch_data_planned(
        ctx: *mut rlnc_context,
        src_dev: *const u8,
        k: usize,
        L: usize,
        num_objects: usize,
        coeffs_dev: *const u8,
        n: usize,
        pieces_dev: *mut u8,
        plan_dev: *const c_void,
    ) -> c_int;
    pub fn rlnc_recode_batch(
        ctx: *mut rlnc_context,
        pieces_dev: *const u8,
        k: usize,
        L: usize,
        n: usize,
        num_objects: usize,
        r_dev: *const u8,
        count: usize,
        out_dev: *mut u8,
    ) -> c_int;
    pub fn rlnc_decode_batch(
        ctx: *mut rlnc_context,
        pieces_dev: *const u8,
        pieces_obj_stride: usize,
        k: usize,
        L: usize,
        m: usize,
        num_objects: usize,
        decoded_dev: *mut u8,
        piece_status: *mut i32,
        object_status: *mut i32,
        data_len: *mut u64,
    ) -> c_int;
    pub fn rlnc_decode_batch_device(
        ctx: *mut rlnc_context,
        pieces_dev: *const u8,
        pieces_obj_stride: usize,
        k: usize,
        L: usize,
        m: usize,
        num_objects: usize,
        decoded_dev: *mut u8,
        piece_status_dev: *mut i32,
        object_status_dev: *mut i32,
        data_len_dev: *mut i64,
    ) -> c_int;
    pub fn rlnc_decode_batch_eliminate(
        ctx: *mut rlnc_context,
        pieces_dev: *const u8,
        pieces_obj_stride: usize,
        k: usize,
        L: usize,
        m: usize,
        num_objects: usize,
        T_dev: *mut u8,
        piece_status_dev: *mut i32,
        rank_dev: *mut i32,
    ) -> c_int;
    pub fn rlnc_decode_batch_apply(
        ctx: *mut rlnc_context,
        pieces_dev: *const u8,
        pieces_obj_stride: usize,
        k: usize,
        L: usize,
        m: usize,
        num_objects: usize,
        T_dev: *const u8,
        rank_dev: *const i32,
        decoded_dev: *mut u8,
        object_status_dev: *mut i32,
        data_len_dev: *mut i64,
    ) -> c_int;
    pub fn rlnc_decode_batch_apply_plan_bytes(k: usize, m: usize, num_objects: usize) -> usize;
    pub fn rlnc_decode_batch_apply_prepare(
        ctx: *mut rlnc_context,
        pieces_dev: *const u8,
        pieces_obj_stride: usize,
        k: usize,
        L: usize,
        m: usize,
        num_objects: usize,
        T_dev: *const u8,
        decoded_dev: *mut u8,
        plan_dev: *mut c_void,
        plan_bytes: usize,
    ) -> c_int;
    pub fn rlnc_decode_batch_apply_planned(
        ctx: *mut rlnc_context,
        pieces_dev: *const u8,
        pieces_obj_stride: usize,
        k: usize,
        L: usize,
        m: usize,
        num_objects: usize,
        T_dev: *const u8,
        rank_dev: *const i32,
        decoded_dev: *mut u8,
        object_status_dev: *mut i32,
        data_len_dev: *mut i64,
        plan_dev: *const c_void,
    ) -> c_int;

    // wire formats on the device
    pub fn rlnc_padded_piece_byte_len(data_len: usize, k: usize) -> usize;
    pub fn rlnc_pad_device(
        ctx: *mut rlnc_context,
        data_dev: *const u8,
        data_len: usize,
        k: usize,
        out_dev: *mut u8,
        out_row_stride: usize,
    ) -> c_int;
    pub fn rlnc_pad_batch_device(ctx: *mut rlnc_context, descs: *const rlnc_pad_desc, count: usize) -> c_int;
    pub fn rlnc_encoder_new_device(
        ctx: *mut rlnc_context,
        data_dev: *const u8,
        data_len: usize,
        piece_count: usize,
        out: *mut *mut rlnc_encoder,
    ) -> c_int;
    pub fn rlnc_encode_ragged(ctx: *mut rlnc_context, objs: *const rlnc_object_desc, count: usize) -> c_int;
    pub fn rlnc_recode_ragged(ctx: *mut rlnc_context, objs: *const rlnc_recode_object_desc, count: usize) -> c_int;
    pub fn rlnc_decode_ragged(
        ctx: *mut rlnc_context,
        objs: *const rlnc_decode_object_desc,
        count: usize,
        piece_status_dev: *mut i32,
        object_status_dev: *mut i32,
        data_len_dev: *mut i64,
    ) -> c_int;

    // host-resident pieces (pinned or pageable host buffers)
    pub fn rlnc_encode_host_stream(
        ctx: *mut rlnc_context,
        src: *const u8,
        k: usize,
        L: usize,
        num_objects: usize,
        coeffs: *const u8,
        n: usize,
        pieces: *mut u8,
        window: usize,
    ) -> c_int;
    pub fn rlnc_decode_host_stream(
        ctx: *mut rlnc_context,
        pieces: *const u8,
        pieces_obj_stride: usize,
        k: usize,
        L: usize,
        m: usize,
        num_objects: usize,
        decoded: *mut u8,
        piece_status: *mut i32,
        object_status: *mut i32,
        data_len: *mut u64,
        window: usize,
    ) -> c_int;

    // host-only exact coefficient elimination (decoder_matrix.rs:99-244 on [coeffs | E])
    pub fn rlnc_elimination_new(k: usize, fixed_slots: usize, out: *mut *mut rlnc_elimination) -> c_int;
    pub fn rlnc_elimination_free(e: *mut rlnc_elimination);
    pub fn rlnc_elimination_push(e: *mut rlnc_elimination, coeffs: *const u8, slot: *mut i32, keep: *mut i32) -> c_int;
    pub fn rlnc_elimination_rank(e: *const rlnc_elimination) -> usize;
    pub fn rlnc_elimination_slots(e: *const rlnc_elimination) -> usize;
    pub fn rlnc_elimination_transform(e: *const rlnc_elimination, T: *mut u8, ld: usize) -> c_int;
    pub fn rlnc_elimination_coefficients(e: *const rlnc_elimination, C: *mut u8) -> c_int;
}
