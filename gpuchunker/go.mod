module github.com/volsync-amd/gpuchunker

// Go 1.18 is the toolchain the restic mover image builds with
// (mover-restic/Dockerfile:2).  The package needs cgo (CGO_ENABLED=1, as the
// image's restic build already uses: mover-restic/Dockerfile:27) and
// libvsgpu.so from ../volsync_amd/lib.
go 1.18
