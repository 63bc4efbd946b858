package gpuchunker

// Tests in the shape of github.com/restic/chunker@v0.4.0 chunker_test.go
// (a reader is chunked with a known polynomial and every chunk's
// Start/Length/Cut/digest is compared with a list), driven by the fixtures
// the Python suite also uses (../tests/golden/cdc_*.json, made by
// tests/golden/make_golden.py).  Needs a GPU: the tests skip when
// DeviceCount() == 0, because the library has no CPU fallback.

import (
	"bytes"
	"crypto/sha256"
	"encoding/binary"
	"encoding/hex"
	"encoding/json"
	"errors"
	"io"
	"os"
	"path/filepath"
	"strconv"
	"strings"
	"testing"
)

// testPol is upstream's chunker_test.go polynomial (degree 53, irreducible).
const testPol = Pol(0x3DA3358B4DC173)

type fixture struct {
	Name  string `json:"name"`
	Input struct {
		Kind      string     `json:"kind"`
		Seed      uint64     `json:"seed"`
		Len       int        `json:"len"`
		Offset    uint64     `json:"offset"`
		Period    int        `json:"period"`
		ZeroRuns  [][2]int   `json:"zero_runs"`
	} `json:"input"`
	Params struct {
		Pol     string `json:"pol"`
		Min     uint   `json:"min"`
		Max     uint   `json:"max"`
		AvgBits int    `json:"avg_bits"`
	} `json:"params"`
	Chunks [][4]json.RawMessage `json:"chunks"`
}

type want struct {
	start, length uint
	cut           uint64
	id            string
}

// synth returns bytes [off, off+n) of the splitmix64 word stream of
// SURVEY.md 8(d) (little-endian u64 words), as oracle/cdc_ref.py synth.
func synth(seed, off uint64, n int) []byte {
	w0 := off >> 3
	w1 := (off + uint64(n) + 7) >> 3
	b := make([]byte, (w1-w0)*8)
	for i := w0; i < w1; i++ {
		z := seed + (i+1)*0x9E3779B97F4A7C15
		z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9
		z = (z ^ (z >> 27)) * 0x94D049BB133111EB
		z ^= z >> 31
		binary.LittleEndian.PutUint64(b[(i-w0)*8:], z)
	}
	a := off - w0*8
	return b[a : a+uint64(n)]
}

func (f *fixture) data(t *testing.T) []byte {
	in := f.Input
	switch in.Kind {
	case "zeros":
		return make([]byte, in.Len)
	case "synth":
		return synth(in.Seed, in.Offset, in.Len)
	case "synth_zero_runs":
		d := synth(in.Seed, 0, in.Len)
		for _, r := range in.ZeroRuns {
			for i := r[0]; i < r[1]; i++ {
				d[i] = 0
			}
		}
		return d
	case "synth_repeat":
		base := synth(in.Seed, 0, in.Period)
		d := make([]byte, 0, in.Len+in.Period)
		for len(d) < in.Len {
			d = append(d, base...)
		}
		return d[:in.Len]
	}
	t.Fatalf("%s: unknown input kind %q", f.Name, in.Kind)
	return nil
}

func parseUint(t *testing.T, raw json.RawMessage) uint64 {
	var s string
	if json.Unmarshal(raw, &s) == nil {
		v, err := strconv.ParseUint(strings.TrimPrefix(s, "0x"), 16, 64)
		if err != nil {
			t.Fatal(err)
		}
		return v
	}
	var v uint64
	if err := json.Unmarshal(raw, &v); err != nil {
		t.Fatal(err)
	}
	return v
}

func (f *fixture) want(t *testing.T) []want {
	w := make([]want, len(f.Chunks))
	for i, c := range f.Chunks {
		var id string
		if err := json.Unmarshal(c[3], &id); err != nil {
			t.Fatal(err)
		}
		w[i] = want{uint(parseUint(t, c[0])), uint(parseUint(t, c[1])), parseUint(t, c[2]), id}
	}
	return w
}

func loadFixtures(t *testing.T) []*fixture {
	paths, err := filepath.Glob(filepath.Join("..", "tests", "golden", "cdc_*.json"))
	if err != nil || len(paths) == 0 {
		t.Fatalf("no fixtures: %v", err)
	}
	var fs []*fixture
	for _, p := range paths {
		b, err := os.ReadFile(p)
		if err != nil {
			t.Fatal(err)
		}
		f := &fixture{}
		if err := json.Unmarshal(b, f); err != nil {
			t.Fatalf("%s: %v", p, err)
		}
		fs = append(fs, f)
	}
	return fs
}

func needGPU(t *testing.T) {
	if DeviceCount() == 0 {
		t.Skip("no MI355X device: libvsgpu has no CPU fallback")
	}
}

// testWithData chunks data and compares against chunks, as upstream's
// testWithData: Start/Length/Cut of every chunk, plus its digest (upstream
// compares sha256 of Data; here also the GPU blob ID).
func testWithData(t *testing.T, name string, ch *Chunker, data []byte, chunks []want) {
	buf := make([]byte, MaxSize)
	for i, w := range chunks {
		c, err := ch.Next(buf)
		if err != nil {
			t.Fatalf("%s: chunk %d: Next: %v", name, i, err)
		}
		if c.Start != w.start || c.Length != w.length || c.Cut != w.cut {
			t.Fatalf("%s: chunk %d: got (%d, %d, %#x), want (%d, %d, %#x)", name, i,
				c.Start, c.Length, c.Cut, w.start, w.length, w.cut)
		}
		if !bytes.Equal(c.Data, data[c.Start:c.Start+c.Length]) {
			t.Fatalf("%s: chunk %d: Data differs from the input bytes", name, i)
		}
		sum := sha256.Sum256(c.Data)
		if hex.EncodeToString(sum[:]) != w.id || c.ID != sum {
			t.Fatalf("%s: chunk %d: blob ID %x, sha256(Data) %x, want %s", name, i, c.ID, sum, w.id)
		}
		if len(c.Data) > 0 && &c.Data[0] != &buf[0] {
			t.Fatalf("%s: chunk %d: Data does not alias the caller's buffer", name, i)
		}
	}
	if _, err := ch.Next(buf); err != io.EOF {
		t.Fatalf("%s: after the last chunk: got %v, want io.EOF", name, err)
	}
}

func TestChunkerFixtures(t *testing.T) {
	needGPU(t)
	for _, f := range loadFixtures(t) {
		var pol Pol
		if err := pol.UnmarshalJSON([]byte(`"` + strings.TrimPrefix(f.Params.Pol, "0x") + `"`)); err != nil {
			t.Fatal(err)
		}
		data := f.data(t)
		ch := NewWithBoundaries(bytes.NewReader(data), pol, f.Params.Min, f.Params.Max)
		ch.SetAverageBits(f.Params.AvgBits)
		testWithData(t, f.Name, ch, data, f.want(t))
		ch.Close()
	}
}

// Upstream's zero-data known answer: 4 MinSize chunks of zeros, Cut 0.
func TestChunkerZeroKAT(t *testing.T) {
	needGPU(t)
	data := make([]byte, 4*MinSize)
	ch := New(bytes.NewReader(data), testPol)
	defer ch.Close()
	id := "07854d2fef297a06ba81685e660c332de36d5d18d546927d30daad6d7fda1541"
	chunks := []want{{0, MinSize, 0, id}, {MinSize, MinSize, 0, id},
		{2 * MinSize, MinSize, 0, id}, {3 * MinSize, MinSize, 0, id}}
	testWithData(t, "zeros", ch, data, chunks)
}

// Reset reuses the device handle for a new stream with the same result.
func TestChunkerReset(t *testing.T) {
	needGPU(t)
	data := synth(1, 0, 8*MiB)
	ch := New(bytes.NewReader(data), testPol)
	defer ch.Close()
	var first []Chunk
	for {
		c, err := ch.Next(nil)
		if err == io.EOF {
			break
		}
		if err != nil {
			t.Fatal(err)
		}
		first = append(first, c)
	}
	ch.Reset(bytes.NewReader(data), testPol)
	for i := range first {
		c, err := ch.Next(nil)
		if err != nil {
			t.Fatal(err)
		}
		if c.Start != first[i].Start || c.Length != first[i].Length || c.Cut != first[i].Cut || c.ID != first[i].ID {
			t.Fatalf("chunk %d differs after Reset", i)
		}
	}
}

func TestChunkerWithoutPolynomial(t *testing.T) {
	ch := New(bytes.NewReader(make([]byte, 1<<20)), 0)
	if _, err := ch.Next(nil); err == nil || err.Error() != errTables.Error() {
		t.Fatalf("got %v, want %q", err, errTables)
	}
}

type failingReader struct{ n int }

var errReader = errors.New("reader failed")

func (r *failingReader) Read(p []byte) (int, error) {
	if r.n <= 0 {
		return 0, errReader
	}
	k := len(p)
	if k > r.n {
		k = r.n
	}
	r.n -= k
	return k, nil
}

// A reader error propagates unchanged out of Next.
func TestReaderErrorPropagates(t *testing.T) {
	needGPU(t)
	ch := New(&failingReader{n: 3 << 20}, testPol)
	defer ch.Close()
	for {
		_, err := ch.Next(nil)
		if err == nil {
			continue
		}
		if err != errReader {
			t.Fatalf("got %v, want the reader's error", err)
		}
		return
	}
}

func TestPolynomials(t *testing.T) {
	if testPol.Deg() != 53 || !testPol.Irreducible() {
		t.Fatalf("testPol: degree %d, irreducible %v", testPol.Deg(), testPol.Irreducible())
	}
	// x^4+x+1 is irreducible; x^4+x^3+x+1 has the root 1
	if !Pol(0x13).Irreducible() || Pol(0x1b).Irreducible() || Pol(0x13).Mul(3) != 0x35 {
		t.Fatal("degree-4 arithmetic")
	}
	q, r := Pol(0x3DA3358B4DC173).DivMod(0x1b)
	if q.Mul(0x1b).Add(r) != 0x3DA3358B4DC173 {
		t.Fatal("DivMod")
	}
	if DeviceCount() > 0 {
		for _, p := range []Pol{testPol, 0x1b, 0x2d, 1 << 53} {
			if libDeg(p) != p.Deg() || libIrreducible(p) != p.Irreducible() {
				t.Fatalf("%v: Go and libvsgpu disagree", p)
			}
		}
	}
	p, err := RandomPolynomial()
	if err != nil || p.Deg() != 53 || !p.Irreducible() {
		t.Fatalf("RandomPolynomial: %v %v", p, err)
	}
}
