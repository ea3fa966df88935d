//! `cargo test --features hip` (on a machine with an MI355X and librlnc_hip.so): the HIP types against the crate's
//! own CPU types (`crate::full::{CpuEncoder, CpuDecoder, CpuRecoder}`, exported by `reference.patch`) fed by two
//! identically seeded RNGs, so both draw the same coefficient bytes through the same `fill_bytes` calls.  Every coded
//! piece, recoded piece, decode status and decoded byte string must be identical.  The ranges follow the crate's
//! property tests (`src/full/tests.rs:11-15`: data 1 KiB..64 KiB, 32..2048 pieces, so piece lengths down to 1 byte).

use super::{Decoder, Encoder, Recoder};
use crate::RLNCError;
use crate::full::{CpuDecoder, CpuEncoder, CpuRecoder};
use rand::rngs::StdRng;
use rand::{Rng, SeedableRng};

fn twin_rngs(seed: u64) -> (StdRng, StdRng) {
    (StdRng::seed_from_u64(seed), StdRng::seed_from_u64(seed))
}

fn random_bytes(rng: &mut StdRng, len: usize) -> Vec<u8> {
    (0..len).map(|_| rng.random()).collect()
}

#[test]
fn handles_are_send_sync_clone_debug() {
    fn check<T: Send + Sync + Clone + core::fmt::Debug>() {}
    check::<Encoder>();
    check::<Decoder>();
    check::<Recoder>();
}

#[test]
fn constructor_errors_follow_the_reference_order() {
    // encoder.rs:86-91, decoder.rs:66-71, recoder.rs:69-80
    assert_eq!(Encoder::new(vec![], 0).err(), Some(RLNCError::DataLengthZero));
    assert_eq!(Encoder::new(vec![1], 0).err(), Some(RLNCError::PieceCountZero));
    assert_eq!(Decoder::new(0, 0).err(), Some(RLNCError::PieceLengthZero));
    assert_eq!(Decoder::new(1, 0).err(), Some(RLNCError::PieceCountZero));
    assert_eq!(Recoder::new(vec![], 0, 0).err(), Some(RLNCError::NotEnoughPiecesToRecode));
    assert_eq!(Recoder::new(vec![1], 0, 0).err(), Some(RLNCError::PieceLengthZero));
    assert_eq!(Recoder::new(vec![1], 1, 0).err(), Some(RLNCError::PieceCountZero));
    assert_eq!(Recoder::new(vec![1], 1, 1).err(), Some(RLNCError::PieceLengthTooShort));
}

#[test]
fn coded_pieces_are_bit_exact() {
    let mut meta = StdRng::seed_from_u64(0x524c_4e43);
    for case in 0..12u64 {
        let len = meta.random_range(1..=(1usize << 16));
        let k = meta.random_range(1..=2048usize);
        let data = random_bytes(&mut meta, len);
        let hip = Encoder::new(data.clone(), k).expect("hip encoder");
        let cpu = CpuEncoder::new(data, k).expect("cpu encoder");
        assert_eq!(hip.get_piece_byte_len(), cpu.get_piece_byte_len());
        assert_eq!(hip.get_full_coded_piece_byte_len(), cpu.get_full_coded_piece_byte_len());
        let (mut ra, mut rb) = twin_rngs(case);
        for _ in 0..4 {
            assert_eq!(hip.code(&mut ra), cpu.code(&mut rb), "case {case}: len {len}, k {k}");
        }
        let mut short = vec![0u8; hip.get_full_coded_piece_byte_len() - 1];
        assert_eq!(hip.code_with_buf(&mut ra, &mut short), Err(RLNCError::InvalidOutputBuffer));
    }
}

#[test]
fn decode_statuses_and_data_are_bit_exact() {
    let mut meta = StdRng::seed_from_u64(7);
    for case in 0..6u64 {
        let len = meta.random_range((1usize << 10)..=(1usize << 16));
        // the top of the crate's range (2048 pieces of 1 KiB: 1-byte pieces) in the first case
        let k = if case == 0 { 2048 } else { meta.random_range(32..=2048usize) };
        let data = random_bytes(&mut meta, if case == 0 { 1 << 10 } else { len });
        let enc = CpuEncoder::new(data.clone(), k).expect("encoder");
        let mut hip = Decoder::new(enc.get_piece_byte_len(), enc.get_piece_count()).expect("hip decoder");
        let mut cpu = CpuDecoder::new(enc.get_piece_byte_len(), enc.get_piece_count()).expect("cpu decoder");
        let mut rng = StdRng::seed_from_u64(100 + case);
        loop {
            let piece = enc.code(&mut rng);
            let (a, b) = (hip.decode(&piece), cpu.decode(&piece));
            assert_eq!(a, b, "case {case}: k {k}");
            assert_eq!(hip.get_useful_piece_count(), cpu.get_useful_piece_count());
            assert_eq!(hip.get_received_piece_count(), cpu.get_received_piece_count());
            if a == Err(RLNCError::ReceivedAllPieces) {
                break;
            }
        }
        assert_eq!(hip.decode(&[0u8; 3]), Err(RLNCError::ReceivedAllPieces));
        let snapshot = hip.clone();
        assert_eq!(hip.get_decoded_data().expect("hip data"), data);
        assert_eq!(cpu.get_decoded_data().expect("cpu data"), data);
        assert_eq!(snapshot.get_decoded_data().expect("clone data"), data);
    }
}

#[test]
fn recoded_pieces_are_bit_exact_and_redundant_recodes_are_rejected() {
    let mut meta = StdRng::seed_from_u64(11);
    for case in 0..6u64 {
        let len = meta.random_range((1usize << 10)..=(1usize << 16));
        let k = meta.random_range(32..=2048usize);
        let n = meta.random_range(2..=1040usize);
        let data = random_bytes(&mut meta, len);
        let enc = CpuEncoder::new(data.clone(), k).expect("encoder");
        let mut rng = StdRng::seed_from_u64(200 + case);
        let coded: Vec<u8> = (0..n).flat_map(|_| enc.code(&mut rng)).collect();
        let full = enc.get_full_coded_piece_byte_len();
        let mut hip = Recoder::new(coded.clone(), full, k).expect("hip recoder");
        let mut cpu = CpuRecoder::new(coded.clone(), full, k).expect("cpu recoder");
        let (mut ra, mut rb) = twin_rngs(300 + case);
        for _ in 0..3 {
            assert_eq!(hip.recode(&mut ra), cpu.recode(&mut rb), "case {case}: k {k}, n {n}");
        }
        // pieces combined only from pieces the decoder has seen carry no new information (full/tests.rs:121-203)
        let mut dec = Decoder::new(enc.get_piece_byte_len(), k).expect("decoder");
        for piece in coded.chunks_exact(full) {
            let _ = dec.decode(piece);
        }
        let seen = dec.get_useful_piece_count();
        if seen < k {
            for _ in 0..4 {
                assert_eq!(dec.decode(&hip.recode(&mut ra)), Err(RLNCError::PieceNotUseful));
            }
        }
    }
}
