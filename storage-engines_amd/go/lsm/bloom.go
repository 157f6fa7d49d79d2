// Package lsm — drop-in replacement for intellect4all/storage-engines lsm/bloom.go.
//
// Same exported API, same semantics, bit-exact results; the filter's bit array lives in MI355X
// HBM and is built / probed by hand-written gfx950 kernels in libseb_bloom.so (C ABI:
// include/seb_bloom.h).  The callers — lsm/sstable_builder.go:30,53,217 (NewBloomFilter, Add,
// Encode) and lsm/sstable.go:129,206 (DecodeBloomFilter, MayContain) — compile unchanged.
//
// Crossings: a cgo call costs tens of ns, about what the reference's whole Add costs, so Add does
// not cross.  It appends the key to a Go-side arena; the first Encode / MayContain after a run of
// Adds hands the arena to the library in one seb_filter_add_batch call (one H2D copy, one build
// launch).  MayContain crosses once per call and is answered on the library's host copy of the
// bits, lock-free (seb_filter_may_contain).
//
// Errors: the Go API has no error returns.  A device that is out of HBM or absent
// (SEB_ERR_NOMEM / SEB_ERR_DEVICE) does not reach the callers: the library builds / probes on its
// host copy of the filter instead (the "cpu_fallback" option, counted by seb_fallback_count, the
// first one logged to stderr), so a flush or compaction worker keeps running where the reference
// would.  Two exceptions panic through libPanic: SEB_ERR_INTERNAL (a rejected launch or a kernel
// fault, i.e. a library bug, which a fallback must not hide), and a filter of more than 64 MiB of
// bits (about 56M keys at 1% FPR, past any memtable flush or compaction output) whose device copy
// is ahead of its host copy, so no correct base for the fallback exists.  libPanic is otherwise
// left for what the reference also panics on (a decoded filter too short for its numBits, sizing
// outside Go's defined range).
//
// Not compiled in this repository's pipeline: no Go toolchain exists in the build image or on
// the GPU box (see DESIGN.md).  storage-engines_amd/harness/sstable_replay.c exercises the C call
// sequence of per-key Adds, and harness/flush_bench.c (bench.py --config flush) times both that
// and this file's buffered pattern.
//
// Build: copy this file over lsm/bloom.go, point the cgo flags at the checkout, `go build`
// (go 1.21 or later: runtime.Pinner).
package lsm

/*
#cgo CFLAGS: -I${SRCDIR}/../../../include
#cgo LDFLAGS: -L${SRCDIR}/../../lib -lseb_bloom -Wl,-rpath,${SRCDIR}/../../lib
#include <stdint.h>
#include <stdlib.h>
#include "seb_bloom.h"
*/
import "C"

import (
	"runtime"
	"sync"
	"sync/atomic"
	"unsafe"
)

const arenaCap = 64 << 20 // hand the arena over once it holds this many key bytes

// BloomFilter is a probabilistic data structure for membership testing.
// (lsm/bloom.go:10-14: bits, numBits, numHashes — held by the library, in HBM and on the host.)
type BloomFilter struct {
	h       *C.seb_filter
	mu      sync.Mutex  // the hand-over of the arena (concurrent first MayContains)
	pending atomic.Bool // Adds not yet handed over
	data    []byte      // Add arena: key bytes back to back
	offs    []uint64    // key offsets, kept only once key lengths differ (klen == -2)
	n       int
	klen    int // the common key length; -1 before the first Add, -2 once lengths differ
}

func libPanic(op string) {
	panic("lsm: BloomFilter." + op + ": " + C.GoString(C.seb_last_error()))
}

func wrap(h *C.seb_filter) *BloomFilter {
	bf := &BloomFilter{h: h, klen: -1}
	runtime.SetFinalizer(bf, func(b *BloomFilter) { C.seb_filter_free(b.h) })
	return bf
}

// NewBloomFilter creates a new bloom filter with optimal parameters (lsm/bloom.go:19).
// expectedKeys: estimated number of keys to insert
// falsePositiveRate: desired false positive rate (e.g., 0.01 for 1%)
func NewBloomFilter(expectedKeys int, falsePositiveRate float64) *BloomFilter {
	h := C.seb_filter_new(C.int64_t(expectedKeys), C.double(falsePositiveRate))
	if h == nil {
		libPanic("New")
	}
	bf := wrap(h)
	if expectedKeys > 0 && expectedKeys*16 <= arenaCap {
		bf.data = make([]byte, 0, expectedKeys*16)
	}
	return bf
}

func strPtr(s string) *C.uint8_t {
	if len(s) == 0 {
		return nil
	}
	return (*C.uint8_t)(unsafe.Pointer(unsafe.StringData(s)))
}

// Add inserts a key into the bloom filter (lsm/bloom.go:70).  The key bytes are appended to the
// filter's arena; the bits are set on the GPU in one launch at the next Encode / MayContain (the
// SSTable builder calls Add once per sorted entry, then Encode at Finish).  Like the reference's
// Add, it must not run concurrently with other calls on the same filter.
func (bf *BloomFilter) Add(key string) {
	if len(key) != bf.klen {
		switch bf.klen {
		case -1:
			bf.klen = len(key)
		case -2:
		default: // the first key of another length: offsets from here on
			bf.offs = make([]uint64, bf.n+1, 2*bf.n+2)
			for i := range bf.offs {
				bf.offs[i] = uint64(i * bf.klen)
			}
			bf.klen = -2
		}
	}
	bf.data = append(bf.data, key...)
	bf.n++
	if bf.klen == -2 {
		bf.offs = append(bf.offs, uint64(len(bf.data)))
	}
	bf.pending.Store(true)
	if len(bf.data) >= arenaCap {
		bf.handOver()
	}
}

// handOver builds the arena's keys into the filter in one seb_filter_add_batch call.  The C side
// copies them to the device inside the call and keeps no pointer to them.
func (bf *BloomFilter) handOver() {
	bf.mu.Lock()
	defer bf.mu.Unlock()
	if !bf.pending.Load() || bf.n == 0 {
		bf.pending.Store(false)
		return
	}
	var pin runtime.Pinner // the seb_keys struct holds Go pointers: pin what they point to
	defer pin.Unpin()
	kb := (*C.seb_keys)(C.malloc(C.size_t(unsafe.Sizeof(C.seb_keys{}))))
	defer C.free(unsafe.Pointer(kb))
	*kb = C.seb_keys{n: C.uint64_t(bf.n)}
	if len(bf.data) > 0 {
		pin.Pin(&bf.data[0])
		kb.data = (*C.uint8_t)(unsafe.Pointer(&bf.data[0]))
	}
	if bf.klen == -2 {
		pin.Pin(&bf.offs[0])
		kb.offsets = (*C.uint64_t)(unsafe.Pointer(&bf.offs[0]))
	} else {
		kb.stride = C.uint32_t(bf.klen)
	}
	if C.seb_filter_add_batch(bf.h, kb) != 0 {
		libPanic("Add")
	}
	bf.data, bf.offs, bf.n, bf.klen = bf.data[:0], nil, 0, -1
	bf.pending.Store(false)
}

// MayContain checks if a key might be in the set (lsm/bloom.go:82).
// Returns true if the key might be present (or false positive)
// Returns false if the key is definitely not present
func (bf *BloomFilter) MayContain(key string) bool {
	if bf.pending.Load() {
		bf.handOver()
	}
	rc := C.seb_filter_may_contain(bf.h, strPtr(key), C.uint64_t(len(key)))
	runtime.KeepAlive(key)
	if rc < 0 {
		libPanic("MayContain")
	}
	return rc == 1
}

// MayContainBatch answers MayContain for many keys in one GPU launch (additive API; a batched
// LSM MultiGet is the intended caller).  out must have len(keys) elements.
func (bf *BloomFilter) MayContainBatch(keys []string, out []bool) {
	if len(out) < len(keys) {
		panic("lsm: MayContainBatch: out too short")
	}
	if len(keys) == 0 {
		return
	}
	if bf.pending.Load() {
		bf.handOver()
	}
	total := 0
	for _, k := range keys {
		total += len(k)
	}
	data := make([]byte, total+1)
	offs := make([]uint64, len(keys)+1)
	pos := 0
	for i, k := range keys {
		offs[i] = uint64(pos)
		pos += copy(data[pos:], k)
	}
	offs[len(keys)] = uint64(pos)
	var pin runtime.Pinner
	defer pin.Unpin()
	pin.Pin(&data[0])
	pin.Pin(&offs[0])
	kb := (*C.seb_keys)(C.malloc(C.size_t(unsafe.Sizeof(C.seb_keys{}))))
	defer C.free(unsafe.Pointer(kb))
	*kb = C.seb_keys{
		data:    (*C.uint8_t)(unsafe.Pointer(&data[0])),
		offsets: (*C.uint64_t)(unsafe.Pointer(&offs[0])),
		n:       C.uint64_t(len(keys)),
	}
	// Go's bool is one byte holding 0 or 1: the library writes exactly that.
	if C.seb_filter_may_contain_batch(bf.h, kb, (*C.uint8_t)(unsafe.Pointer(&out[0]))) != 0 {
		libPanic("MayContainBatch")
	}
}

// Encode serializes the bloom filter to bytes (lsm/bloom.go:96).
// Format: [numBits(8)][numHashes(4)][bits...]
func (bf *BloomFilter) Encode() []byte {
	if bf.pending.Load() {
		bf.handOver()
	}
	n := C.seb_filter_encoded_size(bf.h)
	buf := make([]byte, int(n))
	if C.seb_filter_encode(bf.h, (*C.uint8_t)(unsafe.Pointer(&buf[0])), n) != 0 {
		libPanic("Encode")
	}
	return buf
}

// DecodeBloomFilter deserializes a bloom filter from bytes (lsm/bloom.go:105).
func DecodeBloomFilter(data []byte) *BloomFilter {
	if len(data) < 12 {
		return nil
	}
	h := C.seb_filter_decode((*C.uint8_t)(unsafe.Pointer(&data[0])), C.uint64_t(len(data)))
	runtime.KeepAlive(data)
	if h == nil {
		return nil
	}
	return wrap(h)
}
