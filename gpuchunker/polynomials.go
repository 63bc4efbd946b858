package gpuchunker

// GF(2)[x] polynomial arithmetic: the API of github.com/restic/chunker@v0.4.0
// polynomials.go (SURVEY.md 8(a) row A1).  A Pol is a polynomial over GF(2)
// whose bit i is the coefficient of x^i.  This is host-side arithmetic that
// runs once per repository (restic init), so it stays in Go; the kernels
// only receive the tables built from it (vs_pol_tables, row A2).

import (
	"crypto/rand"
	"encoding/binary"
	"errors"
	"fmt"
	"io"
	"strconv"
	"strings"
)

// Pol is a polynomial from F_2[X].
type Pol uint64

// Add returns x+y (xor in GF(2)).
func (x Pol) Add(y Pol) Pol { return x ^ y }

// mulOverflows reports whether the carry-less product of a and b needs more
// than 64 bits.
func mulOverflows(a, b Pol) bool {
	if a <= 1 || b <= 1 {
		return false
	}
	return a.Deg()+b.Deg() > 63
}

// Mul returns x*y.  It panics when the product does not fit in 64 bits, as
// the upstream implementation does.
func (x Pol) Mul(y Pol) Pol {
	switch {
	case x == 0 || y == 0:
		return 0
	case x == 1:
		return y
	case y == 1:
		return x
	}
	if mulOverflows(x, y) {
		panic("multiplication would overflow uint64")
	}
	var r Pol
	for i := 0; i <= y.Deg(); i++ {
		if y&(1<<uint(i)) != 0 {
			r ^= x << uint(i)
		}
	}
	return r
}

// Deg returns the degree of x, or -1 for the zero polynomial.
func (x Pol) Deg() int {
	d := -1
	for v := uint64(x); v != 0; v >>= 1 {
		d++
	}
	return d
}

// String returns x in hexadecimal.
func (x Pol) String() string { return "0x" + strconv.FormatUint(uint64(x), 16) }

// Expand returns x as a sum of powers, e.g. "x^3+x+1".
func (x Pol) Expand() string {
	if x == 0 {
		return "0"
	}
	var terms []string
	for i := x.Deg(); i >= 0; i-- {
		if x&(1<<uint(i)) == 0 {
			continue
		}
		switch i {
		case 0:
			terms = append(terms, "1")
		case 1:
			terms = append(terms, "x")
		default:
			terms = append(terms, fmt.Sprintf("x^%d", i))
		}
	}
	return strings.Join(terms, "+")
}

// DivMod returns x / d and x mod d.  It panics on division by zero.
func (x Pol) DivMod(d Pol) (Pol, Pol) {
	if d == 0 {
		panic("division by zero")
	}
	if x == 0 {
		return 0, 0
	}
	dd := d.Deg()
	var q Pol
	for x != 0 && x.Deg() >= dd {
		s := uint(x.Deg() - dd)
		q |= 1 << s
		x ^= d << s
	}
	return q, x
}

// Div returns the quotient x / d.
func (x Pol) Div(d Pol) Pol { q, _ := x.DivMod(d); return q }

// Mod returns the remainder x mod d.
func (x Pol) Mod(d Pol) Pol { _, r := x.DivMod(d); return r }

// MulMod returns x*f mod g without overflowing 64 bits (shift-and-add with
// reduction after each step).
func (x Pol) MulMod(f, g Pol) Pol {
	if x == 0 || f == 0 {
		return 0
	}
	a := x.Mod(g)
	var r Pol
	for i := 0; i <= f.Deg(); i++ {
		if f&(1<<uint(i)) != 0 {
			r ^= a
		}
		a <<= 1
		if a.Deg() >= g.Deg() {
			a ^= g
		}
	}
	return r.Mod(g)
}

// GCD returns the greatest common divisor of x and f.
func GCD(x, f Pol) Pol {
	for f != 0 {
		x, f = f, x.Mod(f)
	}
	return x
}

// qp computes x^(2^p) mod g by p squarings of x.
func qp(p uint, g Pol) Pol {
	r := Pol(2)
	for i := uint(0); i < p; i++ {
		r = r.MulMod(r, g)
	}
	return r
}

// Irreducible reports whether x is irreducible (Ben-Or's test: x has no
// factor of degree i <= deg/2, i.e. gcd(x^(2^i) - x, x) == 1 for each such i).
// The product library implements the same test (vs_pol_irreducible); the
// test suite checks that the two agree.
func (x Pol) Irreducible() bool {
	for i := 1; i <= x.Deg()/2; i++ {
		if GCD(x, qp(uint(i), x).Add(2)) != 1 {
			return false
		}
	}
	return true
}

// maxRandomTries bounds RandomPolynomial's search: about 1 in 53 random
// degree-53 polynomials is irreducible, so a million tries never fail in
// practice.
const maxRandomTries = 1e6

// RandomPolynomial returns a random irreducible polynomial of degree 53
// drawn from crypto/rand (what restic init stores as ChunkerPolynomial).
func RandomPolynomial() (Pol, error) { return DerivePolynomial(rand.Reader) }

// DerivePolynomial returns an irreducible polynomial of degree 53 derived
// from the bytes of source.
func DerivePolynomial(source io.Reader) (Pol, error) {
	for i := 0; i < maxRandomTries; i++ {
		var b [8]byte
		if _, err := io.ReadFull(source, b[:]); err != nil {
			return 0, err
		}
		f := Pol(binary.LittleEndian.Uint64(b[:]))
		f &= (1 << 54) - 1 // keep degree <= 53
		f |= (1 << 53) | 1  // exactly degree 53, constant term set
		if f.Irreducible() {
			return f, nil
		}
	}
	return 0, errors.New("unable to find new random irreducible polynomial")
}

// MarshalJSON writes x as a hex string, as restic's repository config does.
func (x Pol) MarshalJSON() ([]byte, error) {
	return []byte(`"` + strconv.FormatUint(uint64(x), 16) + `"`), nil
}

// UnmarshalJSON parses a hex string written by MarshalJSON.
func (x *Pol) UnmarshalJSON(data []byte) error {
	if len(data) < 2 || data[0] != '"' || data[len(data)-1] != '"' {
		return errors.New("invalid string for polynomial")
	}
	n, err := strconv.ParseUint(string(data[1:len(data)-1]), 16, 64)
	if err != nil {
		return err
	}
	*x = Pol(n)
	return nil
}
