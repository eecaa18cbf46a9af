//go:build cgo && rocm

// Package rsyncgpu binds librsg.so (include/rsg.h), the MI355X engine for
// gokrazy/rsync's block-checksum hot path.  It is dropped into the reference
// module as internal/rsyncgpu; the build tag keeps the reference's pure-Go
// code the default (release builds are CGO_ENABLED=0, Makefile:4), and
// rsyncgpu_other.go makes New fail with ErrUnavailable everywhere else.
//
// Entry points and the Go code each replaces:
//
//	BlockSums        generateAndSendSums' per-block loop, internal/receiver/generator.go:325-350
//	                 (Checksum1 + Checksum2, internal/rsyncchecksum/rsyncchecksum.go:29,53)
//	GenerateFiles    the generator's host loop for files that reach it, generator.go:143-350
//	HashSearch       hashSearch's byte loop, internal/sender/match.go:21-230
//	HashSearchBatch  SendFiles' per-file hashSearch calls, internal/sender/sender.go:19-115
//	ReceiveData      receiveData's token loop and whole-file check, internal/receiver/receiver.go:98-188
//	ReceiveDataBatch RecvFiles' per-file receiveData calls, receiver.go:18-188 (the call to use for many files)
//	ShardPlan        the block-range plan of a file list over a node's GPUs (SURVEY §8(e))
//	Node             one process driving several GPUs: BlockSums / GenerateFiles sharded over them
//	FileSums         rsyncchecksum.ReaderChecksum (rsyncchecksum.go:60-66), many files per call
//	SumsStream       the per-block Conn writes of a batch, generator.go:317,341-346 (+ mux, wire.go:28-36)
//
// It cannot be compiled in the image it was written in (no Go toolchain); it
// is written against include/rsg.h exactly and tests/c/abi_conformance.c pins
// the struct layouts cgo sees.
package rsyncgpu

/*
#cgo CFLAGS: -I${SRCDIR}/../../third_party/rsync_amd/include
#cgo LDFLAGS: -L${SRCDIR}/../../third_party/rsync_amd/rsync_amd -lrsg -Wl,-rpath,${SRCDIR}/../../third_party/rsync_amd/rsync_amd
#include <stdlib.h>
#include "rsg.h"
extern int32_t rsgGoWrite(void *user, uint8_t *data, uint64_t len);
*/
import "C"

import (
	"errors"
	"fmt"
	"io"
	"os"
	"runtime"
	"runtime/cgo"
	"unsafe"

	"github.com/gokrazy/rsync"
)

// ErrUnavailable: no engine in this build or no gfx950 device; the caller
// keeps the reference's pure-Go path (the single decision point).
var ErrUnavailable = errors.New("rsyncgpu: MI355X engine unavailable")

// ErrCorrupt is RSG_ERR_CORRUPT, the reference's "file corruption" (receiver.go:171-173).
var ErrCorrupt = errors.New("rsyncgpu: whole-file checksum mismatch")

// Engine wraps one rsg_ctx.  Use one per goroutine that calls it concurrently
// (the loopback generator and sender goroutines of clientmaincmd.go:209-228).
type Engine struct{ ctx *C.rsg_ctx }

// New opens device `device`.  RSG_ERR_NODEV maps to ErrUnavailable.
func New(device int) (*Engine, error) {
	// the shared library must be the one this binding's header describes
	if v := int(C.rsg_abi_version()); v != int(C.RSG_ABI_VERSION) {
		return nil, fmt.Errorf("librsg ABI %d, binding built against %d", v, int(C.RSG_ABI_VERSION))
	}
	var ctx *C.rsg_ctx
	if st := C.rsg_ctx_create(C.int32_t(device), &ctx); st != C.RSG_OK {
		if st == C.RSG_ERR_NODEV {
			return nil, fmt.Errorf("%w: %s", ErrUnavailable, C.GoString(C.rsg_last_error(nil)))
		}
		return nil, fmt.Errorf("rsg_ctx_create: %s (%d)", C.GoString(C.rsg_last_error(nil)), int(st))
	}
	return &Engine{ctx}, nil
}

func (e *Engine) Close() { C.rsg_ctx_destroy(e.ctx) }

func (e *Engine) err(st C.rsg_status) error {
	if st == C.RSG_OK {
		return nil
	}
	msg := C.GoString(C.rsg_last_error(e.ctx))
	if st == C.RSG_ERR_CORRUPT {
		return fmt.Errorf("%w: %s", ErrCorrupt, msg)
	}
	return fmt.Errorf("rsg status %d: %s", int(st), msg)
}

func hostErr(st C.rsg_status) error {
	if st == C.RSG_OK {
		return nil
	}
	return fmt.Errorf("rsg status %d: %s", int(st), C.GoString(C.rsg_last_error(nil)))
}

func cHead(h rsync.SumHead) C.rsg_sum_head {
	return C.rsg_sum_head{count: C.int32_t(h.ChecksumCount), block_len: C.int32_t(h.BlockLength),
		s2len: C.int32_t(h.ChecksumLength), rem: C.int32_t(h.RemainderLength)}
}

func goHead(h C.rsg_sum_head) rsync.SumHead {
	return rsync.SumHead{ChecksumCount: int32(h.count), BlockLength: int32(h.block_len),
		ChecksumLength: int32(h.s2len), RemainderLength: int32(h.rem)}
}

func bytePtr(b []byte) *C.uint8_t {
	if len(b) == 0 {
		return nil
	}
	return (*C.uint8_t)(unsafe.Pointer(&b[0]))
}

// Pinned returns page-locked host memory the caller reads files into: the
// engine then DMAs straight from it (no staging copy).  Release with FreePinned.
func (e *Engine) Pinned(n int) ([]byte, error) {
	var p unsafe.Pointer
	if st := C.rsg_alloc_pinned(e.ctx, C.uint64_t(n), &p); st != C.RSG_OK {
		return nil, e.err(st)
	}
	return unsafe.Slice((*byte)(p), n), nil
}

func (e *Engine) FreePinned(b []byte) error {
	if len(b) == 0 {
		return nil
	}
	return e.err(C.rsg_free_pinned(e.ctx, unsafe.Pointer(&b[0])))
}

// BlockSums replaces the per-block loop of generateAndSendSums for a batch of
// files: heads[i] and the 20-byte records of file i (int32 LE sum1 || sum2[16]),
// contiguous, in file order, starting at record first[i].  blockLen 0 =
// SumSizesSqroot (rsynccommon.go:14-37).
func (e *Engine) BlockSums(files [][]byte, blockLen int32, seed int32) ([]rsync.SumHead, []byte, []uint64, error) {
	n := len(files)
	if n == 0 {
		return nil, nil, nil, nil
	}
	// the descriptors hold Go pointers, so they live in C memory with the
	// file slices pinned for the call
	desc := unsafe.Slice((*C.rsg_file)(C.calloc(C.size_t(n), C.sizeof_rsg_file)), n)
	defer C.free(unsafe.Pointer(&desc[0]))
	var pin runtime.Pinner
	defer pin.Unpin()
	for i, f := range files {
		desc[i].len = C.uint64_t(len(f))
		desc[i].block_len = C.int32_t(blockLen)
		if len(f) > 0 {
			pin.Pin(&f[0])
			desc[i].data = (*C.uint8_t)(unsafe.Pointer(&f[0]))
		}
	}
	heads := make([]C.rsg_sum_head, n)
	first := make([]uint64, n)
	var total C.uint64_t
	if st := C.rsg_plan_block_sums(&desc[0], C.uint64_t(n), &heads[0],
		(*C.uint64_t)(unsafe.Pointer(&first[0])), &total); st != C.RSG_OK {
		return nil, nil, nil, hostErr(st)
	}
	rec := make([]byte, int(total)*C.RSG_RECORD_BYTES)
	if st := C.rsg_block_sums_host(e.ctx, &desc[0], C.uint64_t(n), C.int32_t(seed), bytePtr(rec), total); st != C.RSG_OK {
		return nil, nil, nil, e.err(st)
	}
	out := make([]rsync.SumHead, n)
	for i, h := range heads {
		out[i] = goHead(h)
	}
	return out, rec, first, nil
}

// FileSums returns MD4(file) (seeded=false: rsyncchecksum.ReaderChecksum,
// rsyncchecksum.go:60-66) or MD4(int32_LE(seed) || file) (seeded: the
// transfer's file sum, match.go:52-53, receiver.go:117-120) of every file,
// one GPU lane per file.
func (e *Engine) FileSums(files [][]byte, seeded bool, seed int32) ([][16]byte, error) {
	n := len(files)
	if n == 0 {
		return nil, nil
	}
	desc := unsafe.Slice((*C.rsg_file)(C.calloc(C.size_t(n), C.sizeof_rsg_file)), n)
	defer C.free(unsafe.Pointer(&desc[0]))
	var pin runtime.Pinner
	defer pin.Unpin()
	for i, f := range files {
		desc[i].len = C.uint64_t(len(f))
		if len(f) > 0 {
			pin.Pin(&f[0])
			desc[i].data = (*C.uint8_t)(unsafe.Pointer(&f[0]))
		}
	}
	mode := C.int32_t(C.RSG_FILESUM_PLAIN)
	if seeded {
		mode = C.RSG_FILESUM_SEEDED
	}
	out := make([][16]byte, n)
	if st := C.rsg_file_sums_host(e.ctx, &desc[0], C.uint64_t(n), mode, C.int32_t(seed),
		(*C.uint8_t)(unsafe.Pointer(&out[0][0]))); st != C.RSG_OK {
		return nil, e.err(st)
	}
	return out, nil
}

// Match is one (offset, block index) pair hashSearch passes to matched().
type Match struct {
	Offset int64
	Index  int32
}

func goMatches(ms []C.rsg_match) []Match {
	out := make([]Match, len(ms))
	for i, m := range ms {
		out[i] = Match{Offset: int64(m.offset), Index: int32(m.index)}
	}
	return out
}

// sums flattens head.Sums into the arrays rsg_hash_search_* take.
func sums(head rsync.SumHead) ([]uint32, []byte) {
	sum1 := make([]uint32, len(head.Sums))
	sum2 := make([]byte, 16*len(head.Sums)+1)
	for i, s := range head.Sums {
		sum1[i] = s.Sum1
		copy(sum2[16*i:], s.Sum2[:])
	}
	return sum1, sum2
}

// HashSearch replaces hashSearch's byte loop: the (offset, block index) pairs
// hashSearch would pass to matched(), in order.  targets[k] = targets[k].index
// in the Go targets order (sender.go:60-75), which decides among duplicate
// blocks exactly as the reference's unstable sort did.  The caller then runs
// the reference's own matched()/sendToken for each pair and matched(size, -1).
func (e *Engine) HashSearch(src []byte, head rsync.SumHead, targets []int32, seed int32) ([]Match, error) {
	sum1, sum2 := sums(head)
	h := cHead(head)
	capm := len(src)/max(int(head.BlockLength), 1) + 2
	ms := make([]C.rsg_match, capm)
	var nm C.uint64_t
	var s1p *C.uint32_t
	var tp *C.int32_t
	if len(sum1) > 0 {
		s1p = (*C.uint32_t)(unsafe.Pointer(&sum1[0]))
		tp = (*C.int32_t)(unsafe.Pointer(&targets[0]))
	}
	st := C.rsg_hash_search_host(e.ctx, bytePtr(src), C.uint64_t(len(src)), &h, s1p, bytePtr(sum2), tp,
		C.int32_t(seed), &ms[0], C.uint64_t(capm), &nm)
	if st != C.RSG_OK {
		return nil, e.err(st)
	}
	return goMatches(ms[:nm]), nil
}

// SearchJob is one file of SendFiles' loop (sender.go:19-115) whose sums have
// been read (receiveSums, sender.go:51) and whose targets are built
// (sender.go:60-83).
type SearchJob struct {
	Src     []byte
	Head    rsync.SumHead
	Targets []int32
}

// HashSearchBatch replaces hashSearch (sender.go:90) for several files at
// once: the library pipelines them (file i+1 is scanned on the GPU while file
// i's candidates are walked).  Per-file errors come back in errs; a device
// failure stops the batch and is the returned error.
func (e *Engine) HashSearchBatch(jobs []SearchJob, seed int32) ([][]Match, []error, error) {
	n := len(jobs)
	if n == 0 {
		return nil, nil, nil
	}
	cj := unsafe.Slice((*C.rsg_search_job)(C.calloc(C.size_t(n), C.sizeof_rsg_search_job)), n)
	defer C.free(unsafe.Pointer(&cj[0]))
	var pin runtime.Pinner
	defer pin.Unpin()
	raw := make([][]C.rsg_match, n)
	for i, j := range jobs {
		capm := len(j.Src)/max(int(j.Head.BlockLength), 1) + 2
		raw[i] = make([]C.rsg_match, capm)
		pin.Pin(&raw[i][0])
		cj[i].matches, cj[i].match_cap = &raw[i][0], C.uint64_t(capm)
		cj[i].src_len = C.uint64_t(len(j.Src))
		if len(j.Src) > 0 {
			pin.Pin(&j.Src[0])
			cj[i].src = unsafe.Pointer(&j.Src[0])
		}
		sum1, sum2 := sums(j.Head)
		pin.Pin(&sum2[0])
		cj[i].sum2 = (*C.uint8_t)(unsafe.Pointer(&sum2[0]))
		if len(sum1) > 0 {
			pin.Pin(&sum1[0])
			pin.Pin(&j.Targets[0])
			cj[i].sum1 = (*C.uint32_t)(unsafe.Pointer(&sum1[0]))
			cj[i].targets = (*C.int32_t)(unsafe.Pointer(&j.Targets[0]))
		}
		cj[i].head = cHead(j.Head)
	}
	st := C.rsg_hash_search_batch_host(e.ctx, &cj[0], C.uint64_t(n), C.int32_t(seed))
	out := make([][]Match, n)
	errs := make([]error, n)
	for i := range cj {
		if cj[i].status != C.RSG_OK {
			errs[i] = fmt.Errorf("rsg status %d", int(cj[i].status))
			continue
		}
		out[i] = goMatches(raw[i][:cj[i].n_matches])
	}
	if st != C.RSG_OK && st != C.RSG_ERR_INVALID && st != C.RSG_ERR_TRUNCATED {
		return out, errs, e.err(st)
	}
	return out, errs, nil
}

// ReceiveData replaces receiveData's token loop (receiver.go:122-174): stream
// is everything after the SumHead (tokens, int32 0, the 16-byte sum), basis
// the local file's bytes (nil if none).  Returns the rebuilt file; a sum
// mismatch is ErrCorrupt ("file corruption in %s").
func (e *Engine) ReceiveData(stream []byte, head rsync.SumHead, basis []byte, seed int32) ([]byte, error) {
	h := cHead(head)
	var n, used C.uint64_t
	st := C.rsg_apply_tokens(bytePtr(stream), C.uint64_t(len(stream)), &h, bytePtr(basis), C.uint64_t(len(basis)),
		nil, 0, &n, &used)
	if st != C.RSG_OK && st != C.RSG_ERR_TRUNCATED {
		return nil, hostErr(st)
	}
	out := make([]byte, int(n)+1)
	if st := C.rsg_receive_data(e.ctx, bytePtr(stream), C.uint64_t(len(stream)), &h, bytePtr(basis),
		C.uint64_t(len(basis)), C.int32_t(seed), bytePtr(out), n, &n, &used); st != C.RSG_OK {
		return nil, e.err(st)
	}
	return out[:n], nil
}

// SumsStream replaces the generator's per-block Conn writes for a batch
// (generator.go:317,325-350): [int32 idx] SumHead records per file, already
// split into <= 256 KiB mux messages when mux is set (wire.go:28-36).
func SumsStream(idx []int32, heads []rsync.SumHead, rec []byte, mux bool) ([]byte, error) {
	if len(heads) == 0 {
		return nil, nil
	}
	ch := make([]C.rsg_sum_head, len(heads))
	for i, h := range heads {
		ch[i] = cHead(h)
	}
	var ip *C.int32_t
	if idx != nil {
		ip = (*C.int32_t)(unsafe.Pointer(&idx[0]))
	}
	var n C.uint64_t
	if st := C.rsg_encode_sums(ip, &ch[0], C.uint64_t(len(ch)), bytePtr(rec), 0, nil, 0, &n); st != C.RSG_OK &&
		st != C.RSG_ERR_TRUNCATED {
		return nil, hostErr(st)
	}
	out := make([]byte, int(n)+1)
	if st := C.rsg_encode_sums(ip, &ch[0], C.uint64_t(len(ch)), bytePtr(rec), 0, bytePtr(out), n, &n); st != C.RSG_OK {
		return nil, hostErr(st)
	}
	if !mux {
		return out[:n], nil
	}
	var m C.uint64_t
	C.rsg_mux_frame(bytePtr(out), n, 0, C.RSG_CHUNK_SIZE, nil, 0, &m)
	framed := make([]byte, int(m)+1)
	if st := C.rsg_mux_frame(bytePtr(out), n, 0, C.RSG_CHUNK_SIZE, bytePtr(framed), m, &m); st != C.RSG_OK {
		return nil, hostErr(st)
	}
	return framed[:m], nil
}

// GenerateFiles runs the generator's whole host loop for files that reach
// generateAndSendSums (generator.go:143-350): the engine preads every file
// (io.ReadFull per block, :335), hashes it on the GPU and hands the sums
// stream -- idx, SumHead, records per file, the two -1 phase markers -- to w,
// one Write per batch, mux-framed when mux is set (the caller then writes to
// the MultiplexWriter's underlying writer).  w is reached through the
// exported rsgGoWrite (write_rocm.go) with a cgo.Handle kept in C memory.
func (e *Engine) GenerateFiles(files []*os.File, idx []int32, sizes []int64, seed int32, w io.Writer, mux bool) error {
	if len(files) == 0 {
		return nil
	}
	desc := make([]C.rsg_fd_file, len(files))
	for i, f := range files {
		desc[i] = C.rsg_fd_file{fd: C.int32_t(f.Fd()), idx: C.int32_t(idx[i]), len: C.uint64_t(sizes[i])}
	}
	flags := C.int32_t(C.RSG_GEN_IDX | C.RSG_GEN_TERMINATE)
	if mux {
		flags |= C.RSG_GEN_MUX
	}
	h := cgo.NewHandle(w)
	defer h.Delete()
	user := (*cgo.Handle)(C.malloc(C.size_t(unsafe.Sizeof(h))))
	defer C.free(unsafe.Pointer(user))
	*user = h
	var written C.uint64_t
	st := C.rsg_generate_files_fd(e.ctx, &desc[0], C.uint64_t(len(desc)), C.int32_t(seed), flags,
		C.rsg_write_fn(C.rsgGoWrite), unsafe.Pointer(user), nil, &written)
	runtime.KeepAlive(files)
	return e.err(st)
}

// RecvJob is one file of RecvFiles' loop (receiver.go:18-188): the bytes
// after its SumHead (tokens, int32 0, the 16-byte file sum) and its basis.
type RecvJob struct {
	Stream []byte
	Head   rsync.SumHead
	Basis  []byte // nil: no local file
	Size   int64  // rebuilt size (the file list's length)
}

// ReceiveDataBatch replaces receiveData (receiver.go:98-188) for many files
// at once (rsg_receive_data_batch): tokens applied on host threads, the
// seeded whole-file MD4s of a whole batch hashed together on the GPU (one
// lane per file) while the next batch's tokens are applied.  This is the call
// to use for a transfer with many files; per-file errors (ErrCorrupt for a
// sum mismatch) come back in errs.
func (e *Engine) ReceiveDataBatch(jobs []RecvJob, seed int32) ([][]byte, []error, error) {
	n := len(jobs)
	if n == 0 {
		return nil, nil, nil
	}
	cj := unsafe.Slice((*C.rsg_recv_job)(C.calloc(C.size_t(n), C.sizeof_rsg_recv_job)), n)
	defer C.free(unsafe.Pointer(&cj[0]))
	var pin runtime.Pinner
	defer pin.Unpin()
	outs := make([][]byte, n)
	for i, j := range jobs {
		outs[i] = make([]byte, int(j.Size)+1)
		pin.Pin(&outs[i][0])
		cj[i].out, cj[i].out_cap = (*C.uint8_t)(unsafe.Pointer(&outs[i][0])), C.uint64_t(j.Size)
		if len(j.Stream) > 0 {
			pin.Pin(&j.Stream[0])
			cj[i].tokens = (*C.uint8_t)(unsafe.Pointer(&j.Stream[0]))
		}
		cj[i].tokens_len = C.uint64_t(len(j.Stream))
		if len(j.Basis) > 0 {
			pin.Pin(&j.Basis[0])
			cj[i].basis = (*C.uint8_t)(unsafe.Pointer(&j.Basis[0]))
		}
		cj[i].basis_len = C.uint64_t(len(j.Basis))
		cj[i].head = cHead(j.Head)
	}
	st := C.rsg_receive_data_batch(e.ctx, &cj[0], C.uint64_t(n), C.int32_t(seed))
	errs := make([]error, n)
	for i := range cj {
		switch cj[i].status {
		case C.RSG_OK:
			outs[i] = outs[i][:cj[i].out_len]
		case C.RSG_ERR_CORRUPT:
			errs[i], outs[i] = ErrCorrupt, nil
		default:
			errs[i], outs[i] = fmt.Errorf("rsg status %d", int(cj[i].status)), nil
		}
	}
	if st != C.RSG_OK && st != C.RSG_ERR_INVALID && st != C.RSG_ERR_TRUNCATED && st != C.RSG_ERR_CORRUPT {
		return outs, errs, e.err(st)
	}
	return outs, errs, nil
}

// Piece is one entry of a shard plan (rsg_shard_plan): blocks [B0, B1) of
// file File, bytes [Offset, Offset+Length) of it, hashed by device Rank in
// its batch Batch; Record = global record index of block B0.
type Piece struct {
	File, B0, B1, Offset, Length, Record uint64
	BlockLen                             int32
	Rank, Batch                          int32
}

// ShardPlan cuts a file list's global block sequence into world contiguous,
// byte-balanced ranges and each into nbatch batches (block boundaries only).
// blockLens nil: SumSizesSqroot for every file.  records[q][b] = records of
// rank q's batch b.
func ShardPlan(lengths []int64, blockLens []int32, world, nbatch int) ([]Piece, [][]uint64, error) {
	n := len(lengths)
	ln := make([]C.uint64_t, n+1)
	for i, l := range lengths {
		ln[i] = C.uint64_t(l)
	}
	var bl *C.int32_t
	if blockLens != nil {
		bl = (*C.int32_t)(unsafe.Pointer(&blockLens[0]))
	}
	recs := make([]uint64, world*nbatch+1)
	var np C.uint64_t
	st := C.rsg_shard_plan(&ln[0], bl, C.uint64_t(n), 0, C.int32_t(world), C.int32_t(nbatch), nil, 0, &np,
		(*C.uint64_t)(unsafe.Pointer(&recs[0])))
	if st != C.RSG_OK && st != C.RSG_ERR_TRUNCATED {
		return nil, nil, hostErr(st)
	}
	ps := make([]C.rsg_piece, int(np)+1)
	if st := C.rsg_shard_plan(&ln[0], bl, C.uint64_t(n), 0, C.int32_t(world), C.int32_t(nbatch), &ps[0], np, &np,
		(*C.uint64_t)(unsafe.Pointer(&recs[0]))); st != C.RSG_OK {
		return nil, nil, hostErr(st)
	}
	out := make([]Piece, int(np))
	for i := range out {
		p := ps[i]
		out[i] = Piece{File: uint64(p.file), B0: uint64(p.b0), B1: uint64(p.b1), Offset: uint64(p.offset),
			Length: uint64(p.length), Record: uint64(p.record), BlockLen: int32(p.block_len), Rank: int32(p.rank),
			Batch: int32(p.batch)}
	}
	perRank := make([][]uint64, world)
	for q := range perRank {
		perRank[q] = recs[q*nbatch : (q+1)*nbatch]
	}
	return out, perRank, nil
}

// Node is one process driving several GPUs, the shape of gokr-rsync's
// receiver (one generator goroutine, receiver/do.go:96-98): one Engine per
// device, called from the goroutine that owns the Node.  The file list's
// global block sequence is sharded over the devices; outputs are the
// single-device bytes.
type Node struct {
	Engines []*Engine
	ctxs    **C.rsg_ctx // C array of the engines' contexts
}

// NewNode opens one engine per device ordinal.
func NewNode(devices []int) (*Node, error) {
	nd := &Node{}
	for _, d := range devices {
		e, err := New(d)
		if err != nil {
			nd.Close()
			return nil, err
		}
		nd.Engines = append(nd.Engines, e)
	}
	arr := unsafe.Slice((**C.rsg_ctx)(C.calloc(C.size_t(len(devices)+1), C.size_t(unsafe.Sizeof(uintptr(0))))),
		len(devices)+1)
	for i, e := range nd.Engines {
		arr[i] = e.ctx
	}
	nd.ctxs = &arr[0]
	return nd, nil
}

func (nd *Node) Close() {
	for _, e := range nd.Engines {
		e.Close()
	}
	if nd.ctxs != nil {
		C.free(unsafe.Pointer(nd.ctxs))
		nd.ctxs = nil
	}
	nd.Engines = nil
}

func (nd *Node) err(st C.rsg_status) error { return nd.Engines[0].err(st) }

// CommInit builds the RCCL communicator over the node's devices
// (ncclCommInitAll; engine q = rank q) for the device-resident gather.
func (nd *Node) CommInit() error {
	return nd.err(C.rsg_comm_init_all(nd.ctxs, C.int32_t(len(nd.Engines))))
}

// BlockSums is Engine.BlockSums with the file list sharded over the node's
// devices (rsg_block_sums_host_multi): same heads, records and first indices.
func (nd *Node) BlockSums(files [][]byte, blockLen int32, seed int32) ([]rsync.SumHead, []byte, []uint64, error) {
	n := len(files)
	if n == 0 {
		return nil, nil, nil, nil
	}
	desc := unsafe.Slice((*C.rsg_file)(C.calloc(C.size_t(n), C.sizeof_rsg_file)), n)
	defer C.free(unsafe.Pointer(&desc[0]))
	var pin runtime.Pinner
	defer pin.Unpin()
	for i, f := range files {
		desc[i].len = C.uint64_t(len(f))
		desc[i].block_len = C.int32_t(blockLen)
		if len(f) > 0 {
			pin.Pin(&f[0])
			desc[i].data = (*C.uint8_t)(unsafe.Pointer(&f[0]))
		}
	}
	heads := make([]C.rsg_sum_head, n)
	first := make([]uint64, n)
	var total C.uint64_t
	if st := C.rsg_plan_block_sums(&desc[0], C.uint64_t(n), &heads[0],
		(*C.uint64_t)(unsafe.Pointer(&first[0])), &total); st != C.RSG_OK {
		return nil, nil, nil, hostErr(st)
	}
	rec := make([]byte, int(total)*C.RSG_RECORD_BYTES+1)
	if st := C.rsg_block_sums_host_multi(nd.ctxs, C.int32_t(len(nd.Engines)), &desc[0], C.uint64_t(n),
		C.int32_t(seed), bytePtr(rec), total); st != C.RSG_OK {
		return nil, nil, nil, nd.err(st)
	}
	out := make([]rsync.SumHead, n)
	for i, h := range heads {
		out[i] = goHead(h)
	}
	return out, rec[:int(total)*C.RSG_RECORD_BYTES], first, nil
}

// GenerateFiles is Engine.GenerateFiles with every device reading and
// hashing its byte-balanced range of the file list
// (rsg_generate_files_fd_multi); w receives the same stream, written from
// this goroutine's thread in file-list order (generator.go:20-52).
func (nd *Node) GenerateFiles(files []*os.File, idx []int32, sizes []int64, seed int32, w io.Writer, mux bool) error {
	if len(files) == 0 {
		return nil
	}
	desc := make([]C.rsg_fd_file, len(files))
	for i, f := range files {
		desc[i] = C.rsg_fd_file{fd: C.int32_t(f.Fd()), idx: C.int32_t(idx[i]), len: C.uint64_t(sizes[i])}
	}
	flags := C.int32_t(C.RSG_GEN_IDX | C.RSG_GEN_TERMINATE)
	if mux {
		flags |= C.RSG_GEN_MUX
	}
	h := cgo.NewHandle(w)
	defer h.Delete()
	user := (*cgo.Handle)(C.malloc(C.size_t(unsafe.Sizeof(h))))
	defer C.free(unsafe.Pointer(user))
	*user = h
	var written C.uint64_t
	st := C.rsg_generate_files_fd_multi(nd.ctxs, C.int32_t(len(nd.Engines)), &desc[0], C.uint64_t(len(desc)),
		C.int32_t(seed), flags, C.rsg_write_fn(C.rsgGoWrite), unsafe.Pointer(user), nil, &written)
	runtime.KeepAlive(files)
	return nd.err(st)
}

// HashSearchFile replaces hashSearch's byte loop for a source that is an open
// file, as sendFile has it (sender.go:184-206, fileio.go:31-112): the engine
// reads [0, size) of f itself in windows (rsg_hash_search_fd), each searched
// on the GPU while the next is read; a short read is "file has changed
// mid-transfer".  It also returns the whole-file sum MD4(int32_LE(seed) ||
// source) (match.go:52-53), which the caller writes after matched(size, -1).
func (e *Engine) HashSearchFile(f *os.File, size int64, head rsync.SumHead, targets []int32, seed int32) ([]Match, [16]byte, error) {
	var sum [16]byte
	sum1, sum2 := sums(head)
	h := cHead(head)
	capm := int(size)/max(int(head.BlockLength), 1) + 2
	ms := make([]C.rsg_match, capm)
	var nm C.uint64_t
	var s1p *C.uint32_t
	var tp *C.int32_t
	if len(sum1) > 0 {
		s1p = (*C.uint32_t)(unsafe.Pointer(&sum1[0]))
		tp = (*C.int32_t)(unsafe.Pointer(&targets[0]))
	}
	st := C.rsg_hash_search_fd(e.ctx, C.int32_t(f.Fd()), 0, C.uint64_t(size), &h, s1p, bytePtr(sum2), tp,
		C.int32_t(seed), &ms[0], C.uint64_t(capm), &nm, (*C.uint8_t)(unsafe.Pointer(&sum[0])))
	runtime.KeepAlive(f)
	if st != C.RSG_OK {
		return nil, sum, e.err(st)
	}
	return goMatches(ms[:nm]), sum, nil
}

// FileJob is one source file of SendFiles' loop (sender.go:19-115) that is an
// open file: its sums have been read (receiveSums, sender.go:51) and its
// targets built (sender.go:60-83).  Size is the stat'ed size (sendFile's
// fi.Size()).
type FileJob struct {
	File    *os.File
	Size    int64
	Head    rsync.SumHead
	Targets []int32
}

// HashSearchFiles replaces hashSearch (sender.go:90) for several open files
// (rsg_hash_search_fd_batch): each file is read and searched in windows as
// HashSearchFile does, in job order, while the files' whole-file sums
// MD4(int32_LE(seed) || source) (match.go:52-53), written after each
// file's matched(size, -1), run on host threads side by side -- one serial
// MD4 chain per file, several files at once.  A file shorter than its Size
// fails only its own job ("file has changed mid-transfer", fileio.go:99-104);
// per-file errors come back in errs, a device failure is the returned error.
func (e *Engine) HashSearchFiles(jobs []FileJob, seed int32) ([][]Match, [][16]byte, []error, error) {
	n := len(jobs)
	if n == 0 {
		return nil, nil, nil, nil
	}
	cj := unsafe.Slice((*C.rsg_fd_search_job)(C.calloc(C.size_t(n), C.sizeof_rsg_fd_search_job)), n)
	defer C.free(unsafe.Pointer(&cj[0]))
	csums := unsafe.Slice((*byte)(C.calloc(C.size_t(n), 16)), 16*n)
	defer C.free(unsafe.Pointer(&csums[0]))
	var pin runtime.Pinner
	defer pin.Unpin()
	raw := make([][]C.rsg_match, n)
	for i, j := range jobs {
		capm := int(j.Size)/max(int(j.Head.BlockLength), 1) + 2
		raw[i] = make([]C.rsg_match, capm)
		pin.Pin(&raw[i][0])
		cj[i].matches, cj[i].match_cap = &raw[i][0], C.uint64_t(capm)
		cj[i].fd = C.int32_t(j.File.Fd())
		cj[i].src_len = C.uint64_t(j.Size)
		sum1, sum2 := sums(j.Head)
		pin.Pin(&sum2[0])
		cj[i].sum2 = (*C.uint8_t)(unsafe.Pointer(&sum2[0]))
		if len(sum1) > 0 {
			pin.Pin(&sum1[0])
			pin.Pin(&j.Targets[0])
			cj[i].sum1 = (*C.uint32_t)(unsafe.Pointer(&sum1[0]))
			cj[i].targets = (*C.int32_t)(unsafe.Pointer(&j.Targets[0]))
		}
		cj[i].head = cHead(j.Head)
		cj[i].file_sum = (*C.uint8_t)(unsafe.Pointer(&csums[16*i]))
	}
	st := C.rsg_hash_search_fd_batch(e.ctx, &cj[0], C.uint64_t(n), C.int32_t(seed))
	runtime.KeepAlive(jobs)
	out := make([][]Match, n)
	fsums := make([][16]byte, n)
	errs := make([]error, n)
	for i := range cj {
		if cj[i].status != C.RSG_OK {
			errs[i] = fmt.Errorf("rsg status %d", int(cj[i].status))
			continue
		}
		out[i] = goMatches(raw[i][:cj[i].n_matches])
		copy(fsums[i][:], csums[16*i:16*i+16])
	}
	if st != C.RSG_OK && st != C.RSG_ERR_INVALID && st != C.RSG_ERR_TRUNCATED && st != C.RSG_ERR_IO {
		return out, fsums, errs, e.err(st)
	}
	return out, fsums, errs, nil
}
