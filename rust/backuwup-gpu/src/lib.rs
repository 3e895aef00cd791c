//! backuwup-gpu -- the MI355X (gfx950) dedup front end as drop-ins for the three call sites of
//! backuwup's hot path:
//!
//! | reference call site                                              | here                                  |
//! |------------------------------------------------------------------|---------------------------------------|
//! | `fastcdc::v2020::FastCDC::new(&mmap, min, avg, max)` + iterator  | [`fastcdc::v2020::FastCDC`]           |
//! |   (`client/src/backup/filesystem/dir_packer.rs:254-266`)         |                                       |
//! | `blake3::hash(data).into()` (`dir_packer.rs:286`, `:320`, `:353`)| [`blake3::hash`]                      |
//! | `BlobIndex::is_blob_duplicate` under the packer mutex            | [`Context::index_check_insert`],      |
//! |   (`pack.rs:37`, `blob_index.rs:130-148`)                        | batched: [`Context::submit_host`]     |
//! | one `BlobIndex` across the GPUs of a node (north_star)           | [`Comm`] + [`Context::exchange_dedup`]|
//!
//! A maintainer swaps `use fastcdc::v2020::FastCDC;` for `use backuwup_gpu::fastcdc::v2020::FastCDC;`
//! and `blake3::hash` for `backuwup_gpu::blake3::hash` in `dir_packer.rs`; nothing else changes.
//! The drop-ins run on a pool of contexts over every GPU of the node (`BACKUWUP_GPU_DEVICES`,
//! default all), each thread with a home device, because the reference's calls carry no context.  Each is one synchronous GPU round trip; the
//! batched session ([`Context::submit_host`] / [`Context::wait`] with a shared [`Index`]) is the
//! integration a packer should use ("A backup session").
//!
//! Status: written against `include/backuwup_gpu.h` but NOT COMPILED -- the image this repository
//! is built in has no Rust toolchain.  `tests/test_rust_shim.py` parses every `extern "C"`
//! declaration and `#[repr(C)]` struct below and checks name, arity, pointer depth, constness
//! and integer widths against the C header, so the binding cannot drift from the ABI unseen.
#![allow(non_camel_case_types)]

use std::cell::RefCell;
use std::ffi::CStr;
use std::fmt;
use std::os::raw::{c_char, c_int, c_void};

/// The raw C ABI (`include/backuwup_gpu.h`), one declaration per exported function.
pub mod ffi {
    use std::os::raw::{c_char, c_int, c_void};

    pub const BW_OK: c_int = 0;
    pub const BW_EINVAL: c_int = -1;
    pub const BW_ENOSPC: c_int = -2;
    pub const BW_COALESCE_MAX_MSG: u64 = 65_536;
    pub const BW_EHIP: c_int = -3;
    pub const BW_ENOMEM: c_int = -4;
    pub const BW_ECOLLISION: c_int = -5;
    pub const BW_ESTATE: c_int = -6;
    pub const BW_ECRYPTO: c_int = -7;
    pub const BW_EFORMAT: c_int = -8;
    pub const BW_ECOMM: c_int = -9;
    pub const BW_EAGAIN: c_int = -10;

    pub const BW_F_NO_HASH: u32 = 1;
    pub const BW_F_NO_DEDUP: u32 = 2;
    pub const BW_F_SERIAL_RESOLVE: u32 = 4;
    pub const BW_COMM_ID_BYTES: usize = 128;
    pub const BW_COMM_DEFAULT_TIMEOUT_MS: u32 = 120000;
    pub const BW_PACK_ZSTD_STORE: u32 = 1;

    #[repr(C)]
    pub struct bw_ctx {
        _private: [u8; 0],
    }
    #[repr(C)]
    pub struct bw_index {
        _private: [u8; 0],
    }
    #[repr(C)]
    pub struct bw_comm {
        _private: [u8; 0],
    }

    #[repr(C)]
    #[derive(Clone, Copy, Debug, Default)]
    pub struct bw_chunk {
        pub hash: u64,
        pub offset: u64,
        pub length: u64,
    }

    #[repr(C)]
    #[derive(Clone, Copy, Debug)]
    pub struct bw_blob {
        pub file: u64,
        pub offset: u64,
        pub length: u64,
        pub gear_hash: u64,
        pub digest: [u8; 32],
        pub is_dup: u8,
        pub pad: [u8; 7],
    }

    #[repr(C)]
    #[derive(Clone, Copy, Debug, Default)]
    pub struct bw_params {
        pub min_size: u32,
        pub avg_size: u32,
        pub max_size: u32,
        pub flags: u32,
        pub small_file_threshold: u64,
    }

    #[repr(C)]
    #[derive(Clone, Copy, Debug)]
    pub struct bw_tree {
        pub kind: u32,
        pub flags: u32,
        pub size: u64,
        pub mtime: u64,
        pub ctime: u64,
        pub name: *const u8,
        pub name_len: u64,
        pub children: *const u8,
        pub n_children: u64,
    }

    #[repr(C)]
    #[derive(Clone, Copy, Debug, Default)]
    pub struct bw_stream_shard {
        pub ticket: u64,
        pub first_blob: u64,
        pub n_blobs: u64,
        pub chain_start: u64,
        pub rounds: u32,
        pub pad: u32,
    }

    #[repr(C)]
    #[derive(Clone, Copy, Debug)]
    pub struct bw_tree_blob {
        pub tree: u64,
        pub piece: u64,
        pub length: u64,
        pub hash: [u8; 32],
        pub is_dup: u8,
        pub pad: [u8; 7],
    }

    #[repr(C)]
    #[derive(Clone, Copy, Debug, Default)]
    pub struct bw_packfile {
        pub first_blob: u64,
        pub n_blobs: u64,
        pub offset: u64,
        pub size: u64,
        pub header_len: u64,
    }

    #[repr(C)]
    #[derive(Clone, Copy, Debug, Default)]
    pub struct bw_index_file {
        pub file_num: u32,
        pub pad: u32,
        pub offset: u64,
        pub size: u64,
        pub n_entries: u64,
    }

    /// `fn(user, send, recv, bytes_per_rank)`: deliver `send[r * b ..]` to rank r's `recv[my_rank * b ..]`.
    pub type bw_host_all_to_all =
        Option<unsafe extern "C" fn(user: *mut c_void, send: *const c_void, recv: *mut c_void, bytes_per_rank: u64) -> c_int>;

    #[link(name = "backuwup_amd")]
    extern "C" {
        pub fn bw_params_default(p: *mut bw_params);
        pub fn bw_strerror(rc: c_int) -> *const c_char;

        pub fn bw_create(device: c_int, out: *mut *mut bw_ctx) -> c_int;
        pub fn bw_destroy(ctx: *mut bw_ctx);
        pub fn bw_last_error(ctx: *const bw_ctx) -> *const c_char;
        pub fn bw_set_stream(ctx: *mut bw_ctx, hip_stream: *mut c_void) -> c_int;
        pub fn bw_get_stream(ctx: *mut bw_ctx) -> *mut c_void;

        pub fn bw_fastcdc_chunks(ctx: *mut bw_ctx, src: *const u8, len: u64, min_size: u32, avg_size: u32,
                                 max_size: u32, out: *mut bw_chunk, cap: u64, n_out: *mut u64) -> c_int;
        pub fn bw_fastcdc_chunks_hashed(ctx: *mut bw_ctx, src: *const u8, len: u64, min_size: u32, avg_size: u32,
                                        max_size: u32, out: *mut bw_chunk, cap: u64, n_out: *mut u64,
                                        handle: *mut u64) -> c_int;
        pub fn bw_fastcdc_release(handle: u64);
        pub fn bw_blake3_kept_hits() -> u64;
        pub fn bw_blake3_hash(ctx: *mut bw_ctx, data: *const u8, len: u64, out: *mut u8) -> c_int;
        pub fn bw_blake3_hash_dropin(ctx: *mut bw_ctx, data: *const u8, len: u64, out: *mut u8) -> c_int;
        pub fn bw_blake3_hash_dropin_device(device: c_int, data: *const u8, len: u64, out: *mut u8) -> c_int;
        pub fn bw_blake3_coalesce_stats(device: c_int, batches: *mut u64, messages: *mut u64) -> c_int;
        pub fn bw_blake3_service_faults(device: c_int, abandoned: *mut u64, reclaimed: *mut u64,
                                        recovered: *mut u64) -> c_int;
        pub fn bw_device_count(n: *mut c_int) -> c_int;
        pub fn bw_blake3_hash_many(ctx: *mut bw_ctx, data: *const u8, data_len: u64, offsets: *const u64,
                                   lengths: *const u64, n: u64, out: *mut u8) -> c_int;

        pub fn bw_index_reset(ctx: *mut bw_ctx, capacity_hint: u64) -> c_int;
        pub fn bw_index_seed(ctx: *mut bw_ctx, sorted_digests: *const u8, n: u64) -> c_int;
        pub fn bw_index_check_insert(ctx: *mut bw_ctx, digests: *const u8, n: u64, is_dup: *mut u8) -> c_int;
        pub fn bw_index_size(ctx: *mut bw_ctx, n: *mut u64) -> c_int;
        pub fn bw_index_check(ctx: *mut bw_ctx) -> c_int;
        pub fn bw_index_create(device: c_int, out: *mut *mut bw_index) -> c_int;
        pub fn bw_index_destroy(index: *mut bw_index);
        pub fn bw_attach_index(ctx: *mut bw_ctx, index: *mut bw_index) -> c_int;
        pub fn bw_set_option(ctx: *mut bw_ctx, option: c_int, value: u64) -> c_int;

        pub fn bw_process_files(ctx: *mut bw_ctx, data: *const u8, data_len: u64, file_off: *const u64,
                                file_len: *const u64, n_files: u64, params: *const bw_params, out: *mut bw_blob,
                                cap: u64, n_out: *mut u64) -> c_int;
        pub fn bw_submit_device(ctx: *mut bw_ctx, d_data: *const u8, data_len: u64, file_off: *const u64,
                                file_len: *const u64, n_files: u64, params: *const bw_params, ticket: *mut u64)
                                -> c_int;
        pub fn bw_submit_host(ctx: *mut bw_ctx, data: *const u8, data_len: u64, file_off: *const u64,
                              file_len: *const u64, n_files: u64, params: *const bw_params, ticket: *mut u64) -> c_int;
        pub fn bw_wait(ctx: *mut bw_ctx, ticket: u64, out: *mut bw_blob, cap: u64, n_out: *mut u64) -> c_int;
        pub fn bw_host_register(ptr: *mut c_void, len: u64) -> c_int;
        pub fn bw_host_unregister(ptr: *mut c_void) -> c_int;
        pub fn bw_process_files_device(ctx: *mut bw_ctx, d_data: *const u8, data_len: u64, file_off: *const u64,
                                       file_len: *const u64, n_files: u64, params: *const bw_params) -> c_int;
        pub fn bw_results(ctx: *mut bw_ctx, out: *mut bw_blob, cap: u64, n_out: *mut u64) -> c_int;
        pub fn bw_batch_device_views(ctx: *mut bw_ctx, n_blobs: *mut u64, d_digests: *mut *const u8,
                                     d_is_dup: *mut *mut u8) -> c_int;

        pub fn bw_partition_by_owner(ctx: *mut bw_ctx, d_digests: *const u8, n: u64, n_owners: u32, d_out: *mut u8,
                                     d_perm: *mut u64, h_counts: *mut u64) -> c_int;
        pub fn bw_index_check_insert_device(ctx: *mut bw_ctx, d_digests: *const u8, n: u64, d_is_dup: *mut u8)
                                            -> c_int;
        pub fn bw_scatter_verdicts(ctx: *mut bw_ctx, d_verdict: *const u8, d_perm: *const u64, n: u64,
                                   d_is_dup: *mut u8) -> c_int;
        pub fn bw_batch_views(ctx: *mut bw_ctx, ticket: u64, d_n_blobs: *mut *const u64, d_digests: *mut *const u8,
                              d_is_dup: *mut *mut u8, max_blobs: *mut u64) -> c_int;
        pub fn bw_partition_buckets(ctx: *mut bw_ctx, d_digests: *const u8, d_n: *const u64, max_n: u64, cap: u64,
                                    n_owners: u32, d_buckets: *mut u8, d_perm: *mut u64, d_counts: *mut u64) -> c_int;
        pub fn bw_index_check_insert_buckets(ctx: *mut bw_ctx, d_buckets: *const u8, d_counts: *const u64,
                                             n_src: u32, cap: u64, d_verdicts: *mut u8) -> c_int;
        pub fn bw_scatter_buckets(ctx: *mut bw_ctx, d_verdicts: *const u8, d_perm: *const u64,
                                  d_counts: *const u64, n_owners: u32, cap: u64, d_is_dup: *mut u8) -> c_int;

        pub fn bw_comm_unique_id(id: *mut u8) -> c_int;
        pub fn bw_comm_init(device: c_int, rank: c_int, world: c_int, id: *const u8, out: *mut *mut bw_comm) -> c_int;
        pub fn bw_comm_init_timeout(device: c_int, rank: c_int, world: c_int, id: *const u8, timeout_ms: u32,
                                    out: *mut *mut bw_comm) -> c_int;
        pub fn bw_comm_set_timeout(comm: *mut bw_comm, timeout_ms: u32) -> c_int;
        pub fn bw_comm_status(comm: *const bw_comm) -> c_int;
        pub fn bw_comm_init_host(device: c_int, rank: c_int, world: c_int, fn_: bw_host_all_to_all, user: *mut c_void,
                                 out: *mut *mut bw_comm) -> c_int;
        pub fn bw_comm_init_all(devices: *const c_int, n: c_int, timeout_ms: u32, out: *mut *mut bw_comm) -> c_int;
        pub fn bw_comm_init_local(devices: *const c_int, n: c_int, out: *mut *mut bw_comm) -> c_int;
        pub fn bw_comm_destroy(comm: *mut bw_comm);
        pub fn bw_comm_last_error(comm: *const bw_comm) -> *const c_char;
        pub fn bw_comm_set_capacity(comm: *mut bw_comm, cap: u64) -> c_int;
        pub fn bw_exchange_dedup(ctx: *mut bw_ctx, comm: *mut bw_comm, ticket: u64) -> c_int;
        pub fn bw_comm_progress(comm: *mut bw_comm) -> c_int;
        pub fn bw_stream_window(file_len: u64, rank: c_int, world: c_int, max_size: u32, lo: *mut u64,
                                hi: *mut u64) -> c_int;
        pub fn bw_chunk_stream_shard(ctx: *mut bw_ctx, comm: *mut bw_comm, d_window: *const u8, file_len: u64,
                                     params: *const bw_params, out: *mut bw_stream_shard) -> c_int;

        pub fn bw_tree_serialize(tree: *const bw_tree, next_sibling: *const u8, out: *mut u8, cap: u64,
                                 n_out: *mut u64) -> c_int;
        pub fn bw_tree_blobs(ctx: *mut bw_ctx, trees: *const bw_tree, n: u64, flags: u32, tree_hashes: *mut u8,
                             out: *mut bw_tree_blob, cap: u64, n_out: *mut u64) -> c_int;

        pub fn bw_seal_device(ctx: *mut bw_ctx, prk: *const u8, d_src: *const u8, src_off: *const u64,
                              src_len: *const u64, n: u64, info: *const u8, info_len: u32, nonces: *const u8,
                              d_dst: *mut u8, dst_off: *const u64) -> c_int;
        pub fn bw_open_device(ctx: *mut bw_ctx, prk: *const u8, d_src: *const u8, src_off: *const u64,
                              src_len: *const u64, n: u64, info: *const u8, info_len: u32, nonces: *const u8,
                              d_dst: *mut u8, dst_off: *const u64, ok: *mut u8) -> c_int;
        pub fn bw_seal(ctx: *mut bw_ctx, prk: *const u8, src: *const u8, src_off: *const u64, src_len: *const u64,
                       n: u64, info: *const u8, info_len: u32, nonces: *const u8, dst: *mut u8, dst_off: *const u64)
                       -> c_int;
        pub fn bw_open(ctx: *mut bw_ctx, prk: *const u8, src: *const u8, src_off: *const u64, src_len: *const u64,
                       n: u64, info: *const u8, info_len: u32, nonces: *const u8, dst: *mut u8, dst_off: *const u64,
                       ok: *mut u8) -> c_int;

        pub fn bw_zstd_compress_device(ctx: *mut bw_ctx, d_src: *const u8, src_off: *const u64, src_len: *const u64,
                                       n: u64, d_dst: *mut u8, dst_off: *const u64, frame_len: *mut u64) -> c_int;
        pub fn bw_zstd_compress(ctx: *mut bw_ctx, src: *const u8, src_off: *const u64, src_len: *const u64, n: u64,
                                dst: *mut u8, dst_off: *const u64, frame_len: *mut u64) -> c_int;
        pub fn bw_zstd_submit_device(ctx: *mut bw_ctx, d_src: *const u8, src_off: *const u64, src_len: *const u64,
                                     n: u64, d_dst: *mut u8, dst_off: *const u64, ticket: *mut u64) -> c_int;
        pub fn bw_zstd_wait(ctx: *mut bw_ctx, ticket: u64, frame_len: *mut u64) -> c_int;
        pub fn bw_pack_compress_device(ctx: *mut bw_ctx, d_src: *const u8, src_off: *const u64, src_len: *const u64,
                                       n: u64, frame_len: *mut u64) -> c_int;
        pub fn bw_pack_build_compressed(ctx: *mut bw_ctx, prk: *const u8, hashes: *const u8, kinds: *const u8,
                                        nonces: *const u8, plan: *const bw_packfile, npf: u64, ids: *const u8,
                                        d_out: *mut u8) -> c_int;
        pub fn bw_pack_compress(ctx: *mut bw_ctx, src: *const u8, src_off: *const u64, src_len: *const u64, n: u64,
                                frame_len: *mut u64) -> c_int;
        pub fn bw_pack_build_compressed_host(ctx: *mut bw_ctx, prk: *const u8, hashes: *const u8, kinds: *const u8,
                                             nonces: *const u8, plan: *const bw_packfile, npf: u64, ids: *const u8,
                                             out: *mut u8) -> c_int;
        pub fn bw_zstd_store_size(len: u64) -> u64;
        pub fn bw_pack_plan(payload_len: *const u64, n: u64, flags: u32, out: *mut bw_packfile, cap: u64,
                            n_out: *mut u64, total_bytes: *mut u64) -> c_int;
        pub fn bw_pack_plan_session(digests: *const u8, is_dup: *const u8, payload_len: *const u64, n: u64,
                                    flags: u32, out: *mut bw_packfile, cap: u64, n_out: *mut u64,
                                    total_bytes: *mut u64, n_unique: *mut u64) -> c_int;
        pub fn bw_pack_build_device(ctx: *mut bw_ctx, prk: *const u8, d_src: *const u8, src_off: *const u64,
                                    src_len: *const u64, n: u64, hashes: *const u8, kinds: *const u8,
                                    nonces: *const u8, flags: u32, plan: *const bw_packfile, n_packfiles: u64,
                                    packfile_ids: *const u8, d_out: *mut u8) -> c_int;
        pub fn bw_pack_build(ctx: *mut bw_ctx, prk: *const u8, src: *const u8, src_off: *const u64,
                             src_len: *const u64, n: u64, hashes: *const u8, kinds: *const u8, nonces: *const u8,
                             flags: u32, plan: *const bw_packfile, n_packfiles: u64, packfile_ids: *const u8,
                             out: *mut u8) -> c_int;
        pub fn bw_index_files_build(ctx: *mut bw_ctx, prk: *const u8, entries: *const u8, n: u64,
                                    last_file_num: u32, out: *mut u8, cap: u64, files: *mut bw_index_file,
                                    files_cap: u64, n_files: *mut u64, total_bytes: *mut u64) -> c_int;
        pub fn bw_index_load_files(ctx: *mut bw_ctx, prk: *const u8, data: *const u8, files: *const bw_index_file,
                                   n_files: u64, entries: *mut u8, cap: u64, n_entries: *mut u64,
                                   bad_file: *mut u64) -> c_int;

        pub fn bw_profile_enable(ctx: *mut bw_ctx, on: c_int) -> c_int;
        pub fn bw_profile_read(ctx: *mut bw_ctx, stage_ms: *mut f64, n_batches: *mut u64) -> c_int;
        pub fn bw_profile_intervals(ctx: *mut bw_ctx, stage: c_int, out: *mut f64, cap: u64, n: *mut u64) -> c_int;
        pub fn bw_calibrate_b3(ctx: *mut bw_ctx, ms: f64, out: *mut f64) -> c_int;
    }
}

/// A failed call: the C status and the library's message.  `BW_EINVAL` is where the fastcdc
/// crate would have panicked (parameter ranges); the drop-ins below panic there too.
#[derive(Debug, Clone)]
pub struct Error {
    pub rc: c_int,
    pub msg: String,
}

impl fmt::Display for Error {
    fn fmt(&self, f: &mut fmt::Formatter<'_>) -> fmt::Result {
        let text = unsafe { CStr::from_ptr(ffi::bw_strerror(self.rc)) }.to_string_lossy();
        write!(f, "backuwup_amd error {} ({}): {}", self.rc, text, self.msg)
    }
}

impl std::error::Error for Error {}

pub type Result<T> = std::result::Result<T, Error>;

fn message(p: *const c_char) -> String {
    if p.is_null() {
        String::new()
    } else {
        unsafe { CStr::from_ptr(p) }.to_string_lossy().into_owned()
    }
}

/// One GPU context: streams, workspace and a ring of batches in flight.  Not thread-safe; use one
/// per thread, all attached to one shared [`Index`] (the reference's one `BlobIndex` behind the
/// packer mutex, `packfile/mod.rs:77`).
pub struct Context {
    raw: *mut ffi::bw_ctx,
}

unsafe impl Send for Context {}

/// One blob of a batch, in canonical order (files as given, chunks by offset).
pub type Blob = ffi::bw_blob;

impl Context {
    pub fn new(device: i32) -> Result<Context> {
        let mut raw = std::ptr::null_mut();
        let rc = unsafe { ffi::bw_create(device, &mut raw) };
        if rc != ffi::BW_OK {
            return Err(Error { rc, msg: format!("bw_create(device {device})") });
        }
        Ok(Context { raw })
    }

    fn check(&self, rc: c_int) -> Result<()> {
        if rc == ffi::BW_OK {
            Ok(())
        } else {
            Err(Error { rc, msg: message(unsafe { ffi::bw_last_error(self.raw) }) })
        }
    }

    /// `FastCDC::new(src, min, avg, max).collect::<Vec<_>>()` as (hash, offset, length).
    pub fn fastcdc_chunks(&mut self, src: &[u8], min_size: u32, avg_size: u32, max_size: u32)
                          -> Result<Vec<ffi::bw_chunk>> {
        let shortest = std::cmp::max(std::cmp::min(2 * (min_size / 2), max_size), 1) as usize;
        let mut out = vec![ffi::bw_chunk::default(); src.len() / shortest + 2];
        let mut n = 0u64;
        self.check(unsafe {
            ffi::bw_fastcdc_chunks(self.raw, src.as_ptr(), src.len() as u64, min_size, avg_size, max_size,
                                   out.as_mut_ptr(), out.len() as u64, &mut n)
        })?;
        out.truncate(n as usize);
        Ok(out)
    }

    /// As `fastcdc_chunks`, with every chunk's digest kept under the returned handle for
    /// `blake3_hash` of the chunk slices (release with `ffi::bw_fastcdc_release`).
    pub fn fastcdc_chunks_hashed(&mut self, src: &[u8], min_size: u32, avg_size: u32, max_size: u32)
                                 -> Result<(Vec<ffi::bw_chunk>, u64)> {
        let shortest = std::cmp::max(std::cmp::min(2 * (min_size / 2), max_size), 1) as usize;
        let mut out = vec![ffi::bw_chunk::default(); src.len() / shortest + 2];
        let (mut n, mut kept) = (0u64, 0u64);
        self.check(unsafe {
            ffi::bw_fastcdc_chunks_hashed(self.raw, src.as_ptr(), src.len() as u64, min_size, avg_size, max_size,
                                          out.as_mut_ptr(), out.len() as u64, &mut n, &mut kept)
        })?;
        out.truncate(n as usize);
        Ok((out, kept))
    }

    /// `blake3::hash(data).into()`
    pub fn blake3_hash(&mut self, data: &[u8]) -> Result<[u8; 32]> {
        let mut h = [0u8; 32];
        self.check(unsafe { ffi::bw_blake3_hash(self.raw, data.as_ptr(), data.len() as u64, h.as_mut_ptr()) })?;
        Ok(h)
    }

    /// `blake3::hash(data).into()` through the drop-in entry: a chunk slice of a live
    /// `fastcdc_chunks_hashed` source is answered from its kept digest.  The caller guarantees
    /// those bytes do not change while the handle lives (the `FastCDC` drop-in borrows them).
    pub fn blake3_hash_dropin(&mut self, data: &[u8]) -> Result<[u8; 32]> {
        let mut h = [0u8; 32];
        self.check(unsafe { ffi::bw_blake3_hash_dropin(self.raw, data.as_ptr(), data.len() as u64, h.as_mut_ptr()) })?;
        Ok(h)
    }

    /// `blake3::hash` of `data[offsets[i] .. offsets[i] + lengths[i]]` for every i, in one batch.
    pub fn blake3_hash_many(&mut self, data: &[u8], offsets: &[u64], lengths: &[u64]) -> Result<Vec<[u8; 32]>> {
        assert_eq!(offsets.len(), lengths.len());
        let mut out = vec![[0u8; 32]; offsets.len()];
        self.check(unsafe {
            ffi::bw_blake3_hash_many(self.raw, data.as_ptr(), data.len() as u64, offsets.as_ptr(),
                                     lengths.as_ptr(), offsets.len() as u64, out.as_mut_ptr() as *mut u8)
        })?;
        Ok(out)
    }

    /// `BlobIndex::load` (`blob_index.rs:167-200`): empty the index and seed it with the sorted items.
    pub fn index_seed(&mut self, sorted: &[[u8; 32]]) -> Result<()> {
        self.check(unsafe { ffi::bw_index_reset(self.raw, 2 * sorted.len() as u64) })?;
        self.check(unsafe { ffi::bw_index_seed(self.raw, sorted.as_ptr() as *const u8, sorted.len() as u64) })
    }

    /// `is_blob_duplicate` (`blob_index.rs:130-148`) then insert, for digests in canonical order.
    pub fn index_check_insert(&mut self, digests: &[[u8; 32]]) -> Result<Vec<bool>> {
        let mut dup = vec![0u8; digests.len()];
        self.check(unsafe {
            ffi::bw_index_check_insert(self.raw, digests.as_ptr() as *const u8, digests.len() as u64,
                                       dup.as_mut_ptr())
        })?;
        Ok(dup.into_iter().map(|d| d != 0).collect())
    }

    pub fn attach_index(&mut self, index: &Index) -> Result<()> {
        self.check(unsafe { ffi::bw_attach_index(self.raw, index.raw) })
    }

    /// `process_file` + `add_file_blob` (`dir_packer.rs:231-311`) for files lying back to back in
    /// `data`; the batch is copied to HBM while the previous one computes.  `data` must stay
    /// unchanged until the call returns (pageable) or until [`Context::wait`] (pinned).
    pub fn submit_host(&mut self, data: &[u8], file_off: &[u64], file_len: &[u64], params: &ffi::bw_params)
                       -> Result<u64> {
        assert_eq!(file_off.len(), file_len.len());
        let mut ticket = 0u64;
        self.check(unsafe {
            ffi::bw_submit_host(self.raw, data.as_ptr(), data.len() as u64, file_off.as_ptr(), file_len.as_ptr(),
                                file_off.len() as u64, params, &mut ticket)
        })?;
        Ok(ticket)
    }

    /// The blobs of batch `ticket`, canonical order (blocks until it is done).
    pub fn wait(&mut self, ticket: u64) -> Result<Vec<Blob>> {
        let mut n = 0u64;
        let rc = unsafe { ffi::bw_wait(self.raw, ticket, std::ptr::null_mut(), 0, &mut n) };
        if rc != ffi::BW_OK && rc != ffi::BW_ENOSPC {
            self.check(rc)?;
        }
        let mut out: Vec<Blob> = Vec::with_capacity(n as usize);
        self.check(unsafe { ffi::bw_wait(self.raw, ticket, out.as_mut_ptr(), n, &mut n) })?;
        unsafe { out.set_len(n as usize) };
        Ok(out)
    }

    /// Batch `ticket` (submitted with `BW_F_NO_DEDUP`) through the digest-prefix exchange.
    /// One long file split across the ranks of `comm` (a VM image on every GPU of the node):
    /// `window` is this rank's part of it in HBM, file bytes `[lo, hi)` of
    /// `bw_stream_window(file_len, rank, world, max_size)`.  Returns the batch holding this
    /// rank's final chain and the range of its blobs this rank emits; in rank order the emitted
    /// chunks are `FastCDC::new(file, ..)`'s (dir_packer.rs:254-266).  Follow with
    /// `exchange_dedup(comm, shard.ticket)` and `wait(shard.ticket)`.
    pub fn chunk_stream_shard(&mut self, comm: &Comm, d_window: *const u8, file_len: u64, params: &ffi::bw_params)
                              -> Result<ffi::bw_stream_shard> {
        let mut out = ffi::bw_stream_shard::default();
        self.check(unsafe { ffi::bw_chunk_stream_shard(self.raw, comm.raw, d_window, file_len, params, &mut out) })?;
        Ok(out)
    }

    pub fn exchange_dedup(&mut self, comm: &Comm, ticket: u64) -> Result<()> {
        let rc = unsafe { ffi::bw_exchange_dedup(self.raw, comm.raw, ticket) };
        if rc == ffi::BW_ECOMM {
            return Err(Error { rc, msg: message(unsafe { ffi::bw_comm_last_error(comm.raw) }) });
        }
        self.check(rc)
    }

    pub fn as_raw(&self) -> *mut ffi::bw_ctx {
        self.raw
    }
}

impl Drop for Context {
    fn drop(&mut self) {
        unsafe { ffi::bw_destroy(self.raw) }
    }
}

/// The session's seen-chunk index, shared by every attached context.
pub struct Index {
    raw: *mut ffi::bw_index,
}

unsafe impl Send for Index {}
unsafe impl Sync for Index {}

impl Index {
    pub fn new(device: i32) -> Result<Index> {
        let mut raw = std::ptr::null_mut();
        let rc = unsafe { ffi::bw_index_create(device, &mut raw) };
        if rc != ffi::BW_OK {
            return Err(Error { rc, msg: "bw_index_create".into() });
        }
        Ok(Index { raw })
    }
}

impl Drop for Index {
    fn drop(&mut self) {
        unsafe { ffi::bw_index_destroy(self.raw) }
    }
}

/// The transport of the multi-GPU digest exchange: RCCL over xGMI, or the caller's host all-to-all.
pub struct Comm {
    raw: *mut ffi::bw_comm,
    // the host transport's closure and the world size; the library holds a pointer to it
    _host: Option<Box<(HostTransport, usize)>>,
}

unsafe impl Send for Comm {}

type HostTransport = Box<dyn FnMut(&[u8], &mut [u8], usize) -> bool + Send>;

unsafe extern "C" fn host_trampoline(user: *mut c_void, send: *const c_void, recv: *mut c_void, bytes: u64) -> c_int {
    // never unwind into the library
    let r = std::panic::catch_unwind(std::panic::AssertUnwindSafe(|| {
        let t = &mut *(user as *mut (HostTransport, usize));
        let total = bytes as usize * t.1;
        let s = std::slice::from_raw_parts(send as *const u8, total);
        let r = std::slice::from_raw_parts_mut(recv as *mut u8, total);
        (t.0)(s, r, bytes as usize)
    }));
    match r {
        Ok(true) => 0,
        _ => 1,
    }
}

impl Comm {
    /// Rank 0 draws the id; the caller hands its 128 bytes to every rank by any channel.
    pub fn unique_id() -> Result<[u8; ffi::BW_COMM_ID_BYTES]> {
        let mut id = [0u8; ffi::BW_COMM_ID_BYTES];
        let rc = unsafe { ffi::bw_comm_unique_id(id.as_mut_ptr()) };
        if rc != ffi::BW_OK {
            return Err(Error { rc, msg: "ncclGetUniqueId".into() });
        }
        Ok(id)
    }

    /// RCCL communicator of `world` ranks (waits until every rank joined, at most the default
    /// deadline; a rank that never joins gives BW_ECOMM instead of a hang).
    pub fn rccl(device: i32, rank: i32, world: i32, id: &[u8; ffi::BW_COMM_ID_BYTES]) -> Result<Comm> {
        Self::rccl_with_timeout(device, rank, world, id, ffi::BW_COMM_DEFAULT_TIMEOUT_MS)
    }

    /// As `rccl`, with the deadline of every wait on the peers (like the reference transport's
    /// send timeouts, net_p2p/transport.rs:127-128).
    pub fn rccl_with_timeout(device: i32, rank: i32, world: i32, id: &[u8; ffi::BW_COMM_ID_BYTES],
                             timeout_ms: u32) -> Result<Comm> {
        let mut raw = std::ptr::null_mut();
        let rc = unsafe { ffi::bw_comm_init_timeout(device, rank, world, id.as_ptr(), timeout_ms, &mut raw) };
        if rc != ffi::BW_OK {
            return Err(Error { rc, msg: "bw_comm_init_timeout".into() });
        }
        Ok(Comm { raw, _host: None })
    }

    /// Ok while usable; Err(BW_ECOMM) once a failed or stalled peer made the library abort it.
    pub fn status(&self) -> Result<()> {
        let rc = unsafe { ffi::bw_comm_status(self.raw) };
        if rc != ffi::BW_OK {
            return Err(Error { rc, msg: message(unsafe { ffi::bw_comm_last_error(self.raw) }) });
        }
        Ok(())
    }

    /// The caller's transport: `a2a(send, recv, bytes_per_rank)` delivers `send[r * b ..]` to rank
    /// r's `recv[rank * b ..]` and returns true on success.
    pub fn host(device: i32, rank: i32, world: i32,
                a2a: impl FnMut(&[u8], &mut [u8], usize) -> bool + Send + 'static) -> Result<Comm> {
        let mut state: Box<(HostTransport, usize)> = Box::new((Box::new(a2a), world as usize));
        let user = &mut *state as *mut (HostTransport, usize) as *mut c_void;
        let mut raw = std::ptr::null_mut();
        let rc = unsafe { ffi::bw_comm_init_host(device, rank, world, Some(host_trampoline), user, &mut raw) };
        if rc != ffi::BW_OK {
            return Err(Error { rc, msg: "bw_comm_init_host".into() });
        }
        Ok(Comm { raw, _host: Some(state) })
    }

    /// The ranks of ONE process (`bw_comm_init_local`: an in-process host transport, any devices,
    /// several ranks per device included): rank r on `devices[r]`.  Drive each from its own thread.
    pub fn local(devices: &[i32]) -> Result<Vec<Comm>> {
        let mut raw = vec![std::ptr::null_mut(); devices.len()];
        let rc = unsafe { ffi::bw_comm_init_local(devices.as_ptr(), devices.len() as c_int, raw.as_mut_ptr()) };
        if rc != ffi::BW_OK {
            return Err(Error { rc, msg: "bw_comm_init_local".into() });
        }
        Ok(raw.into_iter().map(|raw| Comm { raw, _host: None }).collect())
    }

    /// The ranks of ONE process over RCCL (`bw_comm_init_all`), one distinct device per rank.
    pub fn all(devices: &[i32], timeout_ms: u32) -> Result<Vec<Comm>> {
        let mut raw = vec![std::ptr::null_mut(); devices.len()];
        let rc = unsafe {
            ffi::bw_comm_init_all(devices.as_ptr(), devices.len() as c_int, timeout_ms, raw.as_mut_ptr())
        };
        if rc != ffi::BW_OK {
            return Err(Error { rc, msg: "bw_comm_init_all".into() });
        }
        Ok(raw.into_iter().map(|raw| Comm { raw, _host: None }).collect())
    }

    /// Obsolete since round 5 (accepted and ignored): the exchange sizes its transfers itself.
    pub fn set_capacity(&mut self, cap: u64) -> Result<()> {
        let rc = unsafe { ffi::bw_comm_set_capacity(self.raw, cap) };
        if rc != ffi::BW_OK {
            return Err(Error { rc, msg: "bw_comm_set_capacity".into() });
        }
        Ok(())
    }

    /// Finish the queued exchanges whose digest counts have arrived; never waits for a peer.
    pub fn progress(&mut self) -> Result<()> {
        let rc = unsafe { ffi::bw_comm_progress(self.raw) };
        if rc != ffi::BW_OK {
            return Err(Error { rc, msg: message(unsafe { ffi::bw_comm_last_error(self.raw) }) });
        }
        Ok(())
    }
}

impl Drop for Comm {
    fn drop(&mut self) {
        unsafe { ffi::bw_comm_destroy(self.raw) }
    }
}

/// One backup session over N ranks of THIS process (the reference packs a backup
/// in one process, `client/src/backup/mod.rs:64`): rank r = a context on `devices[r]` whose private
/// index is rank r's shard of the session's `BlobIndex` (owner = digest[0] >> (8 - log2 N)), and a
/// communicator of `Comm::local` or `Comm::all`.  A batch's files are sharded rank-major (contiguous,
/// balanced by bytes), so canonical order = rank order; each rank's thread chunks + hashes its
/// share (`BW_F_NO_DEDUP`), exchanges its digests (`bw_exchange_dedup`) and waits for its verdicts.
/// `backuwup_amd/session.py` is the same sequence (tested on the GPU at world 2 and 4).
pub struct NodeSession {
    // (dropped in this order: a communicator's destruction finishes its queued exchanges, which use
    // the contexts)
    comms: Vec<Comm>,
    ctxs: Vec<Context>,
    params: ffi::bw_params,
}

impl NodeSession {
    /// `rccl`: RCCL over xGMI (one distinct device per rank); otherwise the in-process transport.
    pub fn new(devices: &[i32], rccl: bool, index_hint: u64, mut params: ffi::bw_params) -> Result<NodeSession> {
        assert!(devices.len().is_power_of_two(), "NodeSession: a power-of-two number of ranks");
        let comms = if rccl { Comm::all(devices, ffi::BW_COMM_DEFAULT_TIMEOUT_MS)? } else { Comm::local(devices)? };
        let mut ctxs = Vec::with_capacity(devices.len());
        for &d in devices {
            let c = Context::new(d)?;
            c.check(unsafe { ffi::bw_index_reset(c.raw, index_hint) })?;
            ctxs.push(c);
        }
        params.flags |= ffi::BW_F_NO_DEDUP;
        Ok(NodeSession { comms, ctxs, params })
    }

    /// Every GPU of the node (`bw_device_count`), RCCL between them.
    pub fn all_devices(index_hint: u64, params: ffi::bw_params) -> Result<NodeSession> {
        let mut n: c_int = 0;
        let rc = unsafe { ffi::bw_device_count(&mut n) };
        if rc != ffi::BW_OK || n < 1 {
            return Err(Error { rc, msg: "bw_device_count".into() });
        }
        let world = 1i32 << (31 - (n as u32).leading_zeros());  // the largest power of two <= n
        NodeSession::new(&(0..world).collect::<Vec<_>>(), true, index_hint, params)
    }

    /// The batch (files `data[file_off[i] .. + file_len[i]]`) through every rank -> blobs in canonical
    /// order, `file` = the index in this batch: `Context::submit_host` + `wait` with the gate spread
    /// over the ranks.
    pub fn process_files(&mut self, data: &[u8], file_off: &[u64], file_len: &[u64]) -> Result<Vec<Blob>> {
        assert_eq!(file_off.len(), file_len.len());
        let n = self.ctxs.len();
        let total: f64 = file_len.iter().map(|&l| l as f64 + 1.0).sum();
        let mut cuts = vec![0usize; n + 1];
        let (mut acc, mut f) = (0.0f64, 0usize);
        for r in 1..n {  // contiguous, balanced by bytes (+1 per file: empty files count too)
            while f < file_len.len() && acc + file_len[f] as f64 + 1.0 <= total * r as f64 / n as f64 {
                acc += file_len[f] as f64 + 1.0;
                f += 1;
            }
            cuts[r] = f;
        }
        cuts[n] = file_len.len();
        let params = self.params;
        let results: Vec<Result<Vec<Blob>>> = std::thread::scope(|sc| {
            let hs: Vec<_> = self.ctxs.iter_mut().zip(self.comms.iter_mut()).enumerate().map(|(r, (c, comm))| {
                let (lo, hi) = (cuts[r], cuts[r + 1]);
                sc.spawn(move || -> Result<Vec<Blob>> {
                    let (a, b) = if hi > lo {
                        (file_off[lo..hi].iter().copied().min().unwrap(),
                         (lo..hi).map(|i| file_off[i] + file_len[i]).max().unwrap())
                    } else {
                        (0, 0)
                    };
                    let offs: Vec<u64> = file_off[lo..hi].iter().map(|&o| o - a).collect();
                    let t = c.submit_host(&data[a as usize..b as usize], &offs, &file_len[lo..hi], &params)?;
                    c.exchange_dedup(comm, t)?;
                    let mut res = c.wait(t)?;
                    for b in res.iter_mut() {
                        b.file += lo as u64;
                    }
                    Ok(res)
                })
            }).collect();
            hs.into_iter().map(|h| h.join().expect("a rank's thread panicked")).collect()
        });
        let mut out = Vec::new();
        for r in results {
            out.extend(r?);
        }
        Ok(out)
    }
}

// The drop-ins' contexts: the reference's calls carry none, and tokio runs one worker thread per
// core (client/src/main.rs:43, 256 on an MI355X node), so the threads share a pool of contexts
// instead of holding one each.  The pool spans every GPU of the node: the devices
// are BACKUWUP_GPU_DEVICES ("all", the default, or a list such as "0,1,2,3"; a device may repeat),
// or the single BACKUWUP_GPU_DEVICE of earlier versions; BACKUWUP_GPU_CONTEXTS contexts per listed
// device (default 16).  Thread k (in order of first use) gets home device k mod n: its FastCDC::new
// takes the first free context from its home slot on (contexts alternate devices, so a thread that
// finds its own device's contexts busy moves to the next device's), and its blake3::hash of a small
// message goes to its home device's hash service.  Files are independent (CDC restarts per file,
// dir_packer.rs:254) and the dedup gate stays the caller's (add_blob), so spreading the calls over
// the devices changes no result.
struct Pool {
    devices: Vec<i32>,
    contexts: Vec<std::sync::Mutex<Context>>,  // context j is on devices[j % devices.len()]
}

static POOL: std::sync::OnceLock<Pool> = std::sync::OnceLock::new();
static NEXT_SLOT: std::sync::atomic::AtomicUsize = std::sync::atomic::AtomicUsize::new(0);
thread_local! {
    static SLOT: RefCell<Option<usize>> = RefCell::new(None);
}

/// The devices the drop-ins use (see above).
pub fn pool_devices() -> Vec<i32> {
    let listed = std::env::var("BACKUWUP_GPU_DEVICES").ok();
    match listed.as_deref().map(str::trim) {
        Some(v) if !v.is_empty() && v != "all" => {
            v.split(',').map(|d| d.trim().parse().expect("BACKUWUP_GPU_DEVICES: device numbers")).collect()
        }
        _ => {
            if listed.is_none() {
                if let Some(d) = std::env::var("BACKUWUP_GPU_DEVICE").ok().and_then(|v| v.parse().ok()) {
                    return vec![d];
                }
            }
            let mut n: c_int = 0;
            let rc = unsafe { ffi::bw_device_count(&mut n) };
            assert!(rc == ffi::BW_OK && n > 0, "no MI355X for backuwup-gpu");
            (0..n).collect()
        }
    }
}

fn pool() -> &'static Pool {
    POOL.get_or_init(|| {
        let devices = pool_devices();
        let per = std::env::var("BACKUWUP_GPU_CONTEXTS").ok().and_then(|v| v.parse().ok()).unwrap_or(16usize).max(1);
        let contexts = (0..per * devices.len())
            .map(|j| std::sync::Mutex::new(Context::new(devices[j % devices.len()]).expect("no MI355X for backuwup-gpu")))
            .collect();
        Pool { devices, contexts }
    })
}

fn home_slot() -> usize {
    SLOT.with(|s| *s.borrow_mut().get_or_insert_with(|| NEXT_SLOT.fetch_add(1, std::sync::atomic::Ordering::Relaxed)))
}

/// The device this thread's small `blake3::hash` calls go to.
fn home_device() -> i32 {
    let p = pool();
    p.devices[home_slot() % p.devices.len()]
}

fn with_default<R>(f: impl FnOnce(&mut Context) -> R) -> R {
    let pool = &pool().contexts;
    let start = home_slot() % pool.len();
    for k in 0..pool.len() {
        if let Ok(mut c) = pool[(start + k) % pool.len()].try_lock() {
            return f(&mut c);
        }
    }
    let mut c = pool[start].lock().unwrap_or_else(|e| e.into_inner());
    f(&mut c)
}

/// Drop-in for the `fastcdc` crate 3.0.3, module `v2020`, as backuwup uses it.
pub mod fastcdc {
    pub mod v2020 {
        pub const MINIMUM_MIN: u32 = 64;
        pub const MINIMUM_MAX: u32 = 1_048_576;
        pub const AVERAGE_MIN: u32 = 256;
        pub const AVERAGE_MAX: u32 = 4_194_304;
        pub const MAXIMUM_MIN: u32 = 1024;
        pub const MAXIMUM_MAX: u32 = 16_777_216;

        /// `fastcdc::v2020::Chunk`
        #[derive(Debug, Clone, Copy, PartialEq, Eq, Hash)]
        pub struct Chunk {
            pub hash: u64,
            pub offset: usize,
            pub length: usize,
        }

        /// `fastcdc::v2020::FastCDC`: the whole source is chunked AND every chunk hashed on the GPU
        /// in one submit at construction (`bw_fastcdc_chunks_hashed`); the iterator replays the cuts
        /// (identical boundaries and `Chunk.hash`), and `blake3::hash(&source[off..off + len])` of a
        /// chunk (dir_packer.rs:262-265 -> :286) is answered from the kept digests with no second
        /// trip to the GPU.  The borrow of `source` guarantees the bytes stay put until `Drop`
        /// releases the digests.
        pub struct FastCDC<'a> {
            source: &'a [u8],
            chunks: std::vec::IntoIter<Chunk>,
            kept: u64,
        }

        impl Drop for FastCDC<'_> {
            fn drop(&mut self) {
                unsafe { crate::ffi::bw_fastcdc_release(self.kept) }
            }
        }

        impl<'a> FastCDC<'a> {
            /// Panics where the crate's `FastCDC::new` asserts (size ranges).
            pub fn new(source: &'a [u8], min_size: u32, avg_size: u32, max_size: u32) -> Self {
                assert!((MINIMUM_MIN..=MINIMUM_MAX).contains(&min_size));
                assert!((AVERAGE_MIN..=AVERAGE_MAX).contains(&avg_size));
                assert!((MAXIMUM_MIN..=MAXIMUM_MAX).contains(&max_size));
                // the crate's cut() reads past max here and panics on most sources; the ABI refuses it
                assert!(avg_size <= max_size, "FastCDC: avg_size > max_size");
                let (cuts, kept) = super::super::with_default(|c| {
                    c.fastcdc_chunks_hashed(source, min_size, avg_size, max_size)
                })
                .expect("GPU chunking failed");
                let chunks: Vec<Chunk> = cuts
                    .iter()
                    .map(|c| Chunk { hash: c.hash, offset: c.offset as usize, length: c.length as usize })
                    .collect();
                FastCDC { source, chunks: chunks.into_iter(), kept }
            }

            pub fn source(&self) -> &'a [u8] {
                self.source
            }
        }

        impl Iterator for FastCDC<'_> {
            type Item = Chunk;
            fn next(&mut self) -> Option<Chunk> {
                self.chunks.next()
            }
        }
    }
}

/// Drop-in for the `blake3` crate 1.3.3's `hash` as backuwup uses it (`hash(data).into()`).
pub mod blake3 {
    /// `blake3::Hash`
    #[derive(Clone, Copy, PartialEq, Eq, Hash, Debug)]
    pub struct Hash([u8; 32]);

    impl Hash {
        pub fn as_bytes(&self) -> &[u8; 32] {
            &self.0
        }
        pub fn to_hex(&self) -> String {
            self.0.iter().map(|b| format!("{b:02x}")).collect()
        }
    }

    impl From<Hash> for [u8; 32] {
        fn from(h: Hash) -> [u8; 32] {
            h.0
        }
    }

    impl From<[u8; 32]> for Hash {
        fn from(b: [u8; 32]) -> Hash {
            Hash(b)
        }
    }

    /// `blake3::hash(input)` -- standard unkeyed BLAKE3, 32-byte output, computed on the GPU.  A
    /// chunk of a live `FastCDC` drop-in is answered from the digest its construction kept (safe
    /// Rust cannot change those bytes while the `FastCDC` borrows them); a small message goes to
    /// the hash service of this thread's home device (no launch per call, no context held while
    /// it waits).  What the service does not take -- a message over 64 KiB, or a call it could not
    /// serve in time (`BW_EAGAIN`: the ticket is cancelled and its slot handed on, later calls are
    /// unaffected) -- is hashed through a pool context's own launch path.  Only a failed GPU (the
    /// launch path's error) ends in a panic: the crate's `hash` has no error to return.
    pub fn hash(input: &[u8]) -> Hash {
        let mut h = [0u8; 32];
        let rc = unsafe {
            crate::ffi::bw_blake3_hash_dropin_device(super::home_device(), input.as_ptr(), input.len() as u64,
                                                     h.as_mut_ptr())
        };
        if rc == crate::ffi::BW_OK {
            return Hash(h);
        }
        // BW_EAGAIN (or any failure of the service path): the message through a pool context
        let len = input.len() as u64;
        let d = super::with_default(|c| c.blake3_hash_many(input, &[0], &[len])).expect("the GPU failed");
        Hash(d[0])
    }
}
