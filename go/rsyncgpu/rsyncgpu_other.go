//go:build !(cgo && rocm)

// Package rsyncgpu: every build without `cgo && rocm` (the reference's
// release builds are CGO_ENABLED=0, Makefile:4) gets this file only.  New
// always fails with ErrUnavailable, so the caller keeps the reference's
// pure-Go checksum code at its single decision point; the other methods are
// never reached.
package rsyncgpu

import (
	"errors"
	"io"
	"os"

	"github.com/gokrazy/rsync"
)

var ErrUnavailable = errors.New("rsyncgpu: MI355X engine unavailable")

var ErrCorrupt = errors.New("rsyncgpu: whole-file checksum mismatch")

type Engine struct{}

type Match struct {
	Offset int64
	Index  int32
}

type SearchJob struct {
	Src     []byte
	Head    rsync.SumHead
	Targets []int32
}

func New(device int) (*Engine, error) { return nil, ErrUnavailable }

func (e *Engine) Close() {}

func (e *Engine) Pinned(n int) ([]byte, error) { return nil, ErrUnavailable }

func (e *Engine) FreePinned(b []byte) error { return ErrUnavailable }

func (e *Engine) BlockSums(files [][]byte, blockLen int32, seed int32) ([]rsync.SumHead, []byte, []uint64, error) {
	return nil, nil, nil, ErrUnavailable
}

func (e *Engine) FileSums(files [][]byte, seeded bool, seed int32) ([][16]byte, error) {
	return nil, ErrUnavailable
}

func (e *Engine) HashSearch(src []byte, head rsync.SumHead, targets []int32, seed int32) ([]Match, error) {
	return nil, ErrUnavailable
}

func (e *Engine) HashSearchBatch(jobs []SearchJob, seed int32) ([][]Match, []error, error) {
	return nil, nil, ErrUnavailable
}

func (e *Engine) ReceiveData(stream []byte, head rsync.SumHead, basis []byte, seed int32) ([]byte, error) {
	return nil, ErrUnavailable
}

func SumsStream(idx []int32, heads []rsync.SumHead, rec []byte, mux bool) ([]byte, error) {
	return nil, ErrUnavailable
}

func (e *Engine) GenerateFiles(files []*os.File, idx []int32, sizes []int64, seed int32, w io.Writer, mux bool) error {
	return ErrUnavailable
}

type RecvJob struct {
	Stream []byte
	Head   rsync.SumHead
	Basis  []byte
	Size   int64
}

func (e *Engine) ReceiveDataBatch(jobs []RecvJob, seed int32) ([][]byte, []error, error) {
	return nil, nil, ErrUnavailable
}

type Piece struct {
	File, B0, B1, Offset, Length, Record uint64
	BlockLen                             int32
	Rank, Batch                          int32
}

func ShardPlan(lengths []int64, blockLens []int32, world, nbatch int) ([]Piece, [][]uint64, error) {
	return nil, nil, ErrUnavailable
}

type Node struct{ Engines []*Engine }

func NewNode(devices []int) (*Node, error) { return nil, ErrUnavailable }

func (nd *Node) Close() {}

func (nd *Node) CommInit() error { return ErrUnavailable }

func (nd *Node) BlockSums(files [][]byte, blockLen int32, seed int32) ([]rsync.SumHead, []byte, []uint64, error) {
	return nil, nil, nil, ErrUnavailable
}

func (nd *Node) GenerateFiles(files []*os.File, idx []int32, sizes []int64, seed int32, w io.Writer, mux bool) error {
	return ErrUnavailable
}

func (e *Engine) HashSearchFile(f *os.File, size int64, head rsync.SumHead, targets []int32, seed int32) ([]Match, [16]byte, error) {
	return nil, [16]byte{}, ErrUnavailable
}

type FileJob struct {
	File    *os.File
	Size    int64
	Head    rsync.SumHead
	Targets []int32
}

func (e *Engine) HashSearchFiles(jobs []FileJob, seed int32) ([][]Match, [][16]byte, []error, error) {
	return nil, nil, nil, ErrUnavailable
}
