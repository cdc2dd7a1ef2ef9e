/*
 * `java gunzip InputFile.gz OutputFile` on the GPU codec: the reference CLI's behaviour
 * (S/gunzip.java:25-111 -- argument checks and messages, the metadata dump, exit status 1 with the
 * message on stderr, the two speed lines) with io.nayuki.deflate.gpu.GzipInputStream underneath,
 * over the reference's MarkableFileInputStream (the inflater ends exactly, the trailer is read from
 * there).  A DataFormatException is not caught, as in the reference (TL;DR 7 of SURVEY.md).
 */
import java.io.File;
import java.io.FileOutputStream;
import java.io.IOException;
import java.io.OutputStream;
import java.time.Instant;
import io.nayuki.deflate.GzipMetadata;
import io.nayuki.deflate.MarkableFileInputStream;
import io.nayuki.deflate.gpu.GzipInputStream;


public final class gunzip {
	
	public static void main(String[] args) {
		String err = run(args);
		if (err == null)
			return;
		System.err.println(err);
		System.exit(1);
	}
	
	
	private static final String[] OS_TEXT = {"FAT filesystem", "Amiga", "VMS", "Unix", "VM/CMS", "Atari TOS",
		"HPFS filesystem", "Macintosh", "Z-System", "CP/M", "TOPS-20", "NTFS filesystem", "QDOS", "Acorn RISCOS",
		"Unknown"};
	
	
	private static void describe(GzipMetadata m) {
		System.err.println("Last modified: " + m.modificationTimeUnixS()
			.map(t -> Instant.EPOCH.plusSeconds(t).toString()).orElse("N/A"));
		int xfl = m.extraFlags();
		System.err.println("Extra flags: " + (xfl == 2 ? "Maximum compression"
			: xfl == 4 ? "Fastest compression" : "Unknown (" + xfl + ")"));
		System.err.println("Operating system: " + OS_TEXT[m.operatingSystem().ordinal()]);
		System.err.println("File mode: " + (m.isFileText() ? "Text" : "Binary"));
		m.extraField().ifPresent(b -> System.err.println("Extra field: " + b.length + " bytes"));
		m.fileName().ifPresent(s -> System.err.println("File name: " + s));
		m.comment().ifPresent(s -> System.err.println("Comment: " + s));
	}
	
	
	// null on success, else the message the reference prints
	private static String run(String[] args) {
		if (args.length != 2)
			return "Usage: java gunzip InputFile.gz OutputFile";
		var src = new File(args[0]);
		var dst = new File(args[1]);
		String bad = !src.exists() ? "Input path does not exist: " + src
			: src.isDirectory() ? "Input path is a directory: " + src
			: dst.isDirectory() ? "Output path is a directory: " + dst : null;
		if (bad != null)
			return bad;
		
		try (var in = new GzipInputStream(new MarkableFileInputStream(src))) {
			describe(in.getMetadata());
			long t0 = System.nanoTime();
			try (OutputStream out = new FileOutputStream(dst)) {
				in.transferTo(out);
			}
			double secs = (System.nanoTime() - t0) / 1.0e9;
			System.err.printf("Input  speed: %.2f MB/s%n", src.length() / 1e6 / secs);
			System.err.printf("Output speed: %.2f MB/s%n", dst.length() / 1e6 / secs);
		} catch (IOException e) {
			return "I/O exception: " + e.getMessage();
		}
		return null;
	}
	
}
