// Package gpuchunker is a drop-in replacement for
// github.com/restic/chunker@v0.4.0 whose rolling fingerprint, cut selection
// and SHA-256 blob IDs run on an MI355X through libvsgpu.so
// (include/vsgpu.h).  The API is the upstream one (New, NewWithBoundaries,
// Reset, ResetWithBoundaries, SetAverageBits, Next, Chunk, Pol); Chunk
// additionally carries ID, the restic blob ID (sha256.Sum256 of Data), so
// restic's FileSaver can hand it to Repository.SaveBlob instead of hashing
// the chunk again (INTEGRATION.md section 1).
//
// The mover image already rewrites restic's imports with sed
// (mover-restic/patch-sources.sh:16-27); one more line of the same kind
// points internal/archiver at this package.
package gpuchunker

/*
#cgo CFLAGS: -I${SRCDIR}/../include
#cgo LDFLAGS: -L${SRCDIR}/../volsync_amd/lib -lvsgpu -Wl,-rpath,${SRCDIR}/../volsync_amd/lib
#include <stdlib.h>
#include "vsgpu.h"
*/
import "C"

import (
	"errors"
	"io"
	"runtime"
	"unsafe"
)

const (
	KiB = 1024
	MiB = 1024 * KiB

	// MinSize is the default minimal size of a chunk (chunker.go MinSize).
	MinSize = 512 * KiB
	// MaxSize is the default maximal size of a chunk (chunker.go MaxSize).
	MaxSize = 8 * MiB

	// readSize is how much of the reader one feed hands to the device.  The
	// upstream chunker reads 512 KiB at a time; the GPU wants large batches
	// (the library pipelines them internally: vs_cdc_set_batch_bytes).
	readSize = 64 * MiB

	// DefaultBatchBytes is the device batch of one Chunker: one read.
	DefaultBatchBytes = readSize
	// DefaultMaxPending bounds the stream bytes a Chunker holds for chunks
	// not yet returned (Chunk.Data).  At the bound Next waits for the blob
	// IDs of batches in flight instead of reading on, so a Chunker holds at
	// most max(maxPending, 2*batch + 2*MaxSize) + readSize bytes of the
	// stream plus its 64 MiB read buffer: 384 MiB with the defaults
	// (INTEGRATION.md, "Host memory per Chunker").  restic runs
	// FileReadConcurrency (2) Chunkers per mover.
	DefaultMaxPending = 4 * DefaultBatchBytes
)

// Chunk is one content-defined chunk of the stream (chunker.go Chunk) plus
// its restic blob ID.
type Chunk struct {
	Start  uint
	Length uint
	Cut    uint64
	Data   []byte
	ID     [32]byte
}

// errTables is the upstream error text for a zero polynomial.
var errTables = errors.New("tables for polynomial computation not initialized")

// Chunker splits a byte stream into content-defined chunks.  Like the
// upstream Chunker it is not safe for concurrent use: restic's FileSaver
// workers each own one (archiver.Options.FileReadConcurrency).
type Chunker struct {
	h        *C.vs_cdc
	rd       io.Reader
	pol      Pol
	min, max uint
	bits     int
	err      error // sticky open/reset error, reported by Next

	pending    []byte // bytes read but not yet returned as Chunk.Data
	maxPending int    // at or above it, Next waits for batches in flight
	origin     uint   // stream offset of pending[0]
	readBuf    []byte
	eof        bool // the reader is exhausted and the final feed was sent
}

func lastErr() error { return errors.New(C.GoString(C.vs_last_error())) }

// New returns a Chunker with the default boundaries (MinSize, MaxSize) and
// 20 average bits.
func New(rd io.Reader, pol Pol) *Chunker { return NewWithBoundaries(rd, pol, MinSize, MaxSize) }

// NewWithBoundaries returns a Chunker with explicit chunk size limits.
func NewWithBoundaries(rd io.Reader, pol Pol, min, max uint) *Chunker {
	c := &Chunker{maxPending: DefaultMaxPending}
	c.ResetWithBoundaries(rd, pol, min, max)
	runtime.SetFinalizer(c, (*Chunker).Close)
	return c
}

// Reset starts a new stream with the default boundaries, reusing the
// device buffers of this Chunker.
func (c *Chunker) Reset(rd io.Reader, pol Pol) { c.ResetWithBoundaries(rd, pol, MinSize, MaxSize) }

// ResetWithBoundaries starts a new stream with explicit boundaries.
func (c *Chunker) ResetWithBoundaries(rd io.Reader, pol Pol, min, max uint) {
	c.rd, c.pol, c.min, c.max, c.bits = rd, pol, min, max, 20
	c.pending, c.origin, c.eof = c.pending[:0], 0, false
	c.configure()
}

// SetAverageBits sets the number of mask bits of the cut test (the average
// chunk size beyond MinSize is 2^averageBits).
func (c *Chunker) SetAverageBits(averageBits int) {
	c.bits = averageBits
	c.configure()
}

func (c *Chunker) configure() {
	c.err = nil
	if c.pol == 0 { // Next reports it, as the upstream chunker does
		return
	}
	var rc C.int
	if c.h == nil {
		rc = C.vs_cdc_open(0, C.uint64_t(c.pol), C.uint32_t(c.min), C.uint32_t(c.max),
			C.uint32_t(c.bits), &c.h)
	} else {
		rc = C.vs_cdc_reset(c.h, C.uint64_t(c.pol), C.uint32_t(c.min), C.uint32_t(c.max),
			C.uint32_t(c.bits))
	}
	if rc < 0 {
		c.err = lastErr()
		return
	}
	if C.vs_cdc_set_batch_bytes(c.h, C.uint64_t(DefaultBatchBytes)) < 0 {
		c.err = lastErr()
	}
}

// SetMaxPending sets the bound on stream bytes held for chunks not yet
// returned (DefaultMaxPending); smaller values trade throughput for memory.
func (c *Chunker) SetMaxPending(bytes int) { c.maxPending = bytes }

// fill reads the next piece of the stream and copies it into the library
// (which never retains Go pointers: cgo pointer rules).
func (c *Chunker) fill() error {
	if c.readBuf == nil {
		c.readBuf = make([]byte, readSize)
	}
	k, err := io.ReadFull(c.rd, c.readBuf)
	if k > 0 {
		c.pending = append(c.pending, c.readBuf[:k]...)
		if C.vs_cdc_feed(c.h, unsafe.Pointer(&c.readBuf[0]), C.size_t(k), 0) < 0 {
			return lastErr()
		}
	}
	switch err {
	case nil:
		return nil
	case io.EOF, io.ErrUnexpectedEOF:
		c.eof = true
		if C.vs_cdc_feed(c.h, nil, 0, 1) < 0 {
			return lastErr()
		}
		return nil
	default:
		return err // reader errors propagate unchanged
	}
}

// Next returns the next chunk of the stream, or io.EOF after the last one.
// Chunk.Data is append(data[:0], chunk bytes...): it aliases and extends
// the caller's buffer, as upstream.
func (c *Chunker) Next(data []byte) (Chunk, error) {
	if c.pol == 0 {
		return Chunk{}, errTables
	}
	if c.err != nil {
		return Chunk{}, c.err
	}
	var out C.vs_chunk
	var n C.size_t
	for {
		// at the bound, wait for a batch in flight rather than read more; with
		// none in flight the held bytes belong to batches whose cuts need more
		// input, so the stream is fed anyway
		var rc C.int
		if len(c.pending) >= c.maxPending {
			rc = C.vs_cdc_next_wait(c.h, &out, 1, &n)
		} else {
			rc = C.vs_cdc_next(c.h, &out, 1, &n)
		}
		if rc == C.VS_EOF {
			return Chunk{}, io.EOF
		}
		if rc < 0 {
			return Chunk{}, lastErr()
		}
		if n == 1 {
			break
		}
		if c.eof {
			return Chunk{}, errors.New("gpuchunker: no chunk after the final feed")
		}
		if err := c.fill(); err != nil {
			return Chunk{}, err
		}
	}
	lo := uint(out.start) - c.origin
	ln := uint(out.length)
	data = append(data[:0], c.pending[lo:lo+ln]...)
	c.pending = c.pending[lo+ln:]
	c.origin = uint(out.start) + ln
	ch := Chunk{Start: uint(out.start), Length: ln, Cut: uint64(out.cut), Data: data}
	copy(ch.ID[:], C.GoBytes(unsafe.Pointer(&out.id[0]), 32))
	return ch, nil
}

// Close releases the device handle.  A Chunker must not be used after Close.
func (c *Chunker) Close() {
	if c.h != nil {
		C.vs_cdc_close(c.h)
		c.h = nil
	}
}

// DeviceCount returns the number of usable MI355X devices (0 without one:
// the mover then runs the unpatched CPU restic binary).
func DeviceCount() int { return int(C.vs_device_count()) }

// degree and irreducibility as the product library computes them; the tests
// check that they agree with the Go arithmetic in polynomials.go.
func libDeg(p Pol) int          { return int(C.vs_pol_deg(C.uint64_t(p))) }
func libIrreducible(p Pol) bool { return C.vs_pol_irreducible(C.uint64_t(p)) == 1 }
